# PMC passes on the K = 100 config-5 shard (3 EM iterations): VALU-active share and L2 hit rate per kernel
export TAG=r5p KEEP_GOING=0
PMC="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE;TCC_HIT_sum TCC_MISS_sum" \
PMC_MATCH="gs_" PMC_ARGS="--topics 100 --events 12500000 --steps 3 --warmup 1 --converge 0" bash scripts/gpu.sh pmc
