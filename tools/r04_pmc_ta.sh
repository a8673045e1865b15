set -e
CONFIGS="3" PATHS="3" COUNTERS="TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE" bash tools/r04_pmc_sq.sh
mv gpurun_out/sq_c3_p3 gpurun_out/ta_c3_p3
CONFIGS="3" PATHS="3" bash tools/r04_pmc_sq.sh
