# PMC passes of C3's two bottoms (records; compact u16 at 8 trees a lane,
# top 8) and the L2 test on the record image
set -o pipefail
TI_TX16=0 bash scripts/kernel_pmc.sh r5i_c3_rec c3 || exit 1
TI_TX16_ILP=8 TI_TX_TOP=8 bash scripts/kernel_pmc.sh r5i_c3_t16 c3 || exit 2
TI_TX16=0 bash scripts/gpu_c3_l2.sh r5i_c3_l2_rec c3 || exit 3
