mkdir -p gpurun_out
for cfg in a b c; do
  r=$(timeout -k 10 200 python bench.py --no-cpu-baseline 2>>gpurun_out/sweep_err.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || exit 1
  echo "$cfg $r"
done
rm -f gpurun_out/host_trace.txt
JPGE_HOST_TRACE=gpurun_out/host_trace.txt timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 > /dev/null 2>>gpurun_out/sweep_err.log || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl9 -o tl -- python3 bench.py --no-cpu-baseline --no-kernel-events --steps 10 > /dev/null 2>&1 || exit 1
python3 tools/timeline.py gpurun_out/tl9 --skip 400 | head -12
