#!/bin/sh
# Fetch the inloc assets (see scripts/fetch_assets.py for the parity map).
exec python3 "$(dirname "$0")/../../scripts/fetch_assets.py" inloc "$@"
