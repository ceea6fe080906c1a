bash scripts/gpu_ckpt_2rank.sh && bash scripts/gpu_multirank_rehearsal.sh
