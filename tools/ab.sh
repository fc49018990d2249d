#!/bin/bash
# Interleaved A/B of bench.py under environment settings, on one box.
# usage: bash tools/ab.sh ROUNDS "LABEL=ENV..." "LABEL=ENV..." ... -- [bench.py args]
#   e.g. bash tools/ab.sh 2 "off=TTD_WGRAD4T=0" "on=TTD_WGRAD4T=1" -- --steps 20 --warmup 5
# Prints "<label> <value> <ms/step>" per run; logs in gpurun_out/ab_<label>_<round>.log.
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$1; shift
arms=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do arms+=("$1"); shift; done
[ "$1" = "--" ] && shift
for r in $(seq 1 "$R"); do
  for a in "${arms[@]}"; do
    label=${a%%=*}; envs=${a#*=}
    [ "$envs" = "$a" ] && envs=""
    env $envs timeout -k 10 240 python3 bench.py "$@" > "gpurun_out/ab_${label}_${r}.log" 2>&1 || { echo "$label failed"; tail -20 "gpurun_out/ab_${label}_${r}.log"; exit 1; }
    tail -1 "gpurun_out/ab_${label}_${r}.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["ms_per_step"])' "$label"
  done
done
