#!/bin/bash
# quick tests + bench + stamps on the in-tree build, then the A/B libraries
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/r02_quick.sh || exit 1
AB_ARGS="--no-cpu --no-pmc --no-api" ROUNDS=${ROUNDS:-1} bash scripts/ab.sh 2>&1 | grep -v "^=="
