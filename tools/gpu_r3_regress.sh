#!/bin/bash
# End-of-session regression sweep of the documented round-3 configurations at HEAD.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/rg_$name.log 2>&1 || { echo "FAILED $name"; tail -30 gpurun_out/rg_$name.log; exit 1; }
  echo "== $name: $(tail -1 gpurun_out/rg_$name.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d.get("validated"))' 2>/dev/null)"
}
run api41 400 python -u bench.py --api --rows-per-gpu 400000000 --steps 3 --warmup 1
run sec48 400 python -u bench.py --api --workload secondary --rows-per-gpu 470000000 --steps 3 --warmup 1
run ipc2 400 python -u bench.py --gpus 2 --one-gpu --exchange ipc --rows-per-gpu 300000000 --steps 3 --warmup 1
run snappy41 400 python -u bench.py --api --api-codec snappy --rows-per-gpu 400000000 --steps 3 --warmup 1
timeout -k 10 400 python -u benchmarks/run_configs.py netmerger --gb 2 --maps 64 --reducers 1 > gpurun_out/rg_netmerger.json 2> gpurun_out/rg_netmerger.err \
  || { echo "FAILED netmerger"; tail -20 gpurun_out/rg_netmerger.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/rg_netmerger.json'))
print('== netmerger', {k: v for k, v in d.items() if k.endswith('gbps')})"
