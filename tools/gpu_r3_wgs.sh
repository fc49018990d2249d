export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 30 --warmup 5 > gpurun_out/b_wgs_$name.json 2> gpurun_out/b_wgs_$name.err || { tail -5 gpurun_out/b_wgs_$name.err; exit 1; }
  tail -1 gpurun_out/b_wgs_$name.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['ms_per_step'])"
}
for r in a b; do
run base$r TTD_X=0
run wgs64$r TTD_WGRAD_WGS=64
run wgs96$r TTD_WGRAD_WGS=96
run wgs128$r TTD_WGRAD_WGS=128
run wgs160$r TTD_WGRAD_WGS=160
done
