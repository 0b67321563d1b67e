bash scripts/gpu_check.sh && bash scripts/sweep.sh
