set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_r01 -o run -- python3 bench.py --steps 100 --warmup 8 --no-cpu-baseline > gpurun_out/prof_r01.log 2>&1
echo rc=$?
