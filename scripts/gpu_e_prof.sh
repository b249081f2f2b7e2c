bash scripts/gpu_e_emul.sh && bash scripts/prof_lb_fused.sh
