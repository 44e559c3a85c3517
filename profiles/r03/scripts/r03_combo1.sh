bash scripts/r03_frames_diag.sh && bash scripts/r03_pipe_ab.sh
