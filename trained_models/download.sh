#!/bin/sh
# Fetch the models assets (see scripts/fetch_assets.py for the parity map).
exec python3 "$(dirname "$0")/../scripts/fetch_assets.py" models "$@"
