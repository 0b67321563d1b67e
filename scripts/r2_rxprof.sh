#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/pmc_passes.sh r2_c3_l6b scripts/explicit_sweep.py --configs c3 --settings rexplicit:8 --steps 2 || exit $?
scripts/pmc_passes.sh r2_c4_l6b scripts/explicit_sweep.py --configs c4 --settings rexplicit:8 --steps 2 || exit $?
scripts/pmc_passes.sh r2_c4_l4 scripts/explicit_sweep.py --configs c4 --settings bexplicit:4 --steps 2 || exit $?
