# one-off GPU call: TA / TCP / TD counters of k_files_md5 over the alignment variants of
# tools/files_align_probe.py (raw, a16, a16m, a4m, a8m; 1 warm + 3 timed launches each),
# one counter group per pass
set -o pipefail
OUT=gpurun_out
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
export PROBE_REPS=3
i=0
for ctrs in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
            "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum" \
            "TD_TD_BUSY_sum TD_TC_STALL_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $ROOT/$OUT/fa_pmc/p$i -o run -- \
    python3 $ROOT/tools/files_align_probe.py > $ROOT/$OUT/fa_pmc_p$i.log 2>&1 || { tail -5 $ROOT/$OUT/fa_pmc_p$i.log; exit 1; }
done
echo passes-done
