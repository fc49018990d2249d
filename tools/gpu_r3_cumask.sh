export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 30 --warmup 5 > gpurun_out/b_cm_$name.json 2> gpurun_out/b_cm_$name.err || { tail -5 gpurun_out/b_cm_$name.err; exit 1; }
  tail -1 gpurun_out/b_cm_$name.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['ms_per_step'])"
}
run base TTD_X=0
run cus64 TTD_SIDE_CUS=64
run cus96 TTD_SIDE_CUS=96
run cus128 TTD_SIDE_CUS=128
run cus160 TTD_SIDE_CUS=160
run cus128_wgs128 TTD_SIDE_CUS=128 TTD_WGRAD_WGS=128
run wgs128 TTD_WGRAD_WGS=128
run wgs192 TTD_WGRAD_WGS=192
run base2 TTD_X=0
