mkdir -p gpurun_out
for cfg in "4 2 1" "5 2 1" "6 2 1" "8 2 1" "4 3 1" "4 2 2" "6 2 1" "4 2 1"; do set -- $cfg
  res=$(JPGE_LANES=$1 JPGE_LOOKAHEAD=$2 JPGE_DRAIN_LAG=$3 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 2>>gpurun_out/sweep_err.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d['step_ms'], d['host_cpu']['cpus_used'])") || exit 1
  echo "lanes=$1 L=$2 D=$3 $res"
done
