#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash scripts/r04_probe6.sh; bash scripts/r04_probe7.sh
