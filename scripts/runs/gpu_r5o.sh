# PMC passes: C3-f64 on the compact u16 bottom (the new default), C3 per-lane walk
set -o pipefail
bash scripts/kernel_pmc.sh r5o_c3_f64_t16 c3_f64 || exit 1
TI_TX16_PERLANE=1 bash scripts/kernel_pmc.sh r5o_c3_perlane c3 || exit 2
