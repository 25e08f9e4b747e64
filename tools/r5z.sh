#!/bin/bash
# round-5 final (after the shared circular index change): 1m_quality profile + PMC, then the bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/r5v.sh || exit $?
bash tools/r5u.sh || exit $?
