bash scripts/gpu_check.sh && bash scripts/profile.sh
