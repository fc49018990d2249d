export TMPDIR=/tmp
mkdir -p gpurun_out
 timeout -k 10 240 python bench.py --steps 30 --warmup 5 --graph 0 > gpurun_out/b3_eager.json 2>/dev/null || exit 1
tail -1 gpurun_out/b3_eager.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('eager', d['ms_per_step'])"
 timeout -k 10 240 python bench.py --steps 30 --warmup 5 --graph 1 > gpurun_out/b3_seg.json 2>/dev/null || exit 1
tail -1 gpurun_out/b3_seg.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('seg', d['ms_per_step'])"
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 240 python bench.py --steps 30 --warmup 5 --graph 1 > gpurun_out/b3_seg_pc0.json 2>/dev/null || exit 1
tail -1 gpurun_out/b3_seg_pc0.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('seg_pc0', d['ms_per_step'])"
 timeout -k 10 240 python bench.py --steps 30 --warmup 5 --graph 0 > gpurun_out/b3_eager_b.json 2>/dev/null || exit 1
tail -1 gpurun_out/b3_eager_b.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('eager_b', d['ms_per_step'])"
 timeout -k 10 240 python bench.py --steps 30 --warmup 5 --graph 1 > gpurun_out/b3_seg_b.json 2>/dev/null || exit 1
tail -1 gpurun_out/b3_seg_b.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('seg_b', d['ms_per_step'])"
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 240 python bench.py --steps 30 --warmup 5 --graph 1 > gpurun_out/b3_seg_pc0_b.json 2>/dev/null || exit 1
tail -1 gpurun_out/b3_seg_pc0_b.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('seg_pc0_b', d['ms_per_step'])"
