#!/bin/bash
# round-5 final evidence, one call: profile + PMC + suite (r5s), then quality profile + bench lines (r5z)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/r5s.sh || exit $?
bash tools/r5z.sh || exit $?
