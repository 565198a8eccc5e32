set -o pipefail
mkdir -p gpurun_out
for n in 1000000 100000000; do
AGX_STAMPS=1 timeout -k 10 200 python tools/perf.py --n $n --steps 4 --reps 2 > gpurun_out/stamps_$n.log 2>&1 || exit 1
done
timeout -k 10 200 python tools/perf.py --n 1000000 --steps 100 --reps 5 --prof > gpurun_out/perf_1m.json 2>&1 || exit 1
