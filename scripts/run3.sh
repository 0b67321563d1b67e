bash scripts/gpu_check.sh && KB_LIST="40 53 64 80" bash scripts/sweep.sh
