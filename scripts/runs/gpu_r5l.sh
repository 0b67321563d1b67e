# C4 hot-prefix cache: PMC passes at TI_HX_HOT=0 and 16 (where do 2x go?)
set -o pipefail
TI_HX_HOT=0 bash scripts/kernel_pmc.sh r5l_c4_hot0 c4 || exit 1
TI_HX_HOT=16 bash scripts/kernel_pmc.sh r5l_c4_hot16 c4 || exit 2
