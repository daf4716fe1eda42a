# default nxec_encode_objects (tail arena written whole): side-stream copy beside the
# in-place kernel vs the kernel's own last-stripe path (NXEC_FILES_COPY=kernel)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_encode_md5.py -x -q --timeout 120 --timeout-method thread -k "object" > gpurun_out/t_copy.log 2>&1 || { tail -30 gpurun_out/t_copy.log; exit 1; }
tail -1 gpurun_out/t_copy.log
timeout -k 10 300 python3 tools/files_mix_probe.py full10 ragged mix > gpurun_out/files_copy_side.log 2>&1 || exit 1
NXEC_FILES_COPY=kernel timeout -k 10 300 python3 tools/files_mix_probe.py full10 ragged mix > gpurun_out/files_copy_kernel.log 2>&1 || exit 1
cat gpurun_out/files_copy_side.log; echo "-- NXEC_FILES_COPY=kernel"; cat gpurun_out/files_copy_kernel.log
