# host path A/B (TI_HOST_REGISTER) and the headline alone under rocprofv3
set -o pipefail
timeout -k 10 300 python scripts/host_register_ab.py > gpurun_out/r5q_host_register_ab.jsonl 2> gpurun_out/r5q_host_register_ab.err || exit 1
bash scripts/gpu_headline_prof.sh r5q || exit 2
