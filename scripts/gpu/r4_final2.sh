#!/bin/bash
# r4_final2.sh: r4_final.sh (GPU suite, bench lines, step kernel trace) followed by the step PMC passes
cd "$GRAFT_REPO_ROOT" || exit 2
bash scripts/gpu/r4_final.sh || exit $?
bash scripts/gpu/r4_pmc_step.sh || exit $?
echo done
