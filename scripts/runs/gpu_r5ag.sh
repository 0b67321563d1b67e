#!/bin/bash
# C3 occupancy sensitivity: the u16 compact-bottom kernel at one workgroup per
# CU (TI_LX_WGS=1: 1 wave per SIMD, same 8-tree stages) against the default two
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/env_sweep.sh r5ag c3 "TI_LX_WGS=1" "TI_TX16_ILP=4" "TI_TX16_ILP=4 TI_LX_WGS=1"
