#!/bin/bash
# Round-3 closing evidence: full GPU suite + frame rows + default bench line,
# then smoke(), the driver's bench invocation twice and 1024^3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash scripts/r03_full.sh ${1:-r03_s2_final}/full || exit $?
bash scripts/r03_headline.sh ${1:-r03_s2_final}/head || exit $?
