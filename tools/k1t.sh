set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/k1t
timeout -k 10 60 ./jpgenc_amd/bin/k1/k1_base 3840 2160 16 20 90 > gpurun_out/k1t/base.txt 2>&1 || exit 1
cat gpurun_out/k1t/base.txt
timeout -k 10 60 ./jpgenc_amd/bin/k1/k1_stamps 3840 2160 16 5 90 > gpurun_out/k1t/stamps.txt 2>&1 || exit 1
cat gpurun_out/k1t/stamps.txt
JPGE_BENCH_THREADS=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --d2h-steps 0 --steps 10 --solo-batches 1 > gpurun_out/k1t/bench.json 2> gpurun_out/k1t/bench.err || exit 1
grep threads gpurun_out/k1t/bench.err
