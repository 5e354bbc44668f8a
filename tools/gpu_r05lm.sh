bash tools/gpu_r05m.sh && bash tools/gpu_r05l.sh
