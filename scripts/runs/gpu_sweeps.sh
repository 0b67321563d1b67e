# round-4 sweeps after the cover order, then the C3 family's PMC passes
set -o pipefail
P=r4d
bash scripts/env_sweep.sh ${P}_c4 c4 "TI_HX_TOP=7" "TI_HX_TOP=9" "TI_HX_STAGE=4" "TI_HX_ILP=4 TI_HX_STAGE=4" || exit 1
bash scripts/env_sweep.sh ${P}_c3m c3_maxbin "TI_TX_TOP=5" "TI_TX_TOP=7" "TI_LX_ILP=7" || exit 2
bash scripts/env_sweep.sh ${P}_c3 c3 "TI_TX_TOP=5" "TI_TX_TOP=7" "TI_LX_ILP=4" || exit 3
bash scripts/gpu_pmc.sh $P c3 c3_f64 c3_maxbin || exit 4
