# kernel + memory-copy trace of the files bench: where the step's time beyond k_files_md5 goes
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/ftrace -o run -- \
  python3 bench.py --workload files --steps 5 --warmup 1 --no-cpu-baseline --no-host-inclusive > gpurun_out/ftrace.json 2> gpurun_out/ftrace.err || exit 1
ls gpurun_out/ftrace
