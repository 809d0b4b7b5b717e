#!/bin/sh
# Fetch the ivd assets (see scripts/fetch_assets.py for the parity map).
exec python3 "$(dirname "$0")/../../scripts/fetch_assets.py" ivd "$@"
