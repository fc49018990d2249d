#!/bin/bash
# eager vs segmented graph, with and without the side-stream projection shortcuts (fewer joins = fewer segments)
export TMPDIR=/tmp
mkdir -p gpurun_out
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['config'].get('hipgraph_capture'))" $1 $2; }
for i in 1 2; do
timeout -k 10 200 python bench.py > gpurun_out/gab_e$i.log 2>&1 && ms gpurun_out/gab_e$i.log eager &&
timeout -k 10 200 python bench.py --graph 1 > gpurun_out/gab_g$i.log 2>&1 && ms gpurun_out/gab_g$i.log graph &&
TTD_FWD_PROJ_SIDE=0 TTD_CD_SIDE=0 timeout -k 10 200 python bench.py > gpurun_out/gab_en$i.log 2>&1 && ms gpurun_out/gab_en$i.log eager_noproj &&
TTD_FWD_PROJ_SIDE=0 TTD_CD_SIDE=0 timeout -k 10 200 python bench.py --graph 1 > gpurun_out/gab_gn$i.log 2>&1 && ms gpurun_out/gab_gn$i.log graph_noproj &&
TTD_FWD_PROJ_SIDE=0 timeout -k 10 200 python bench.py --graph 1 > gpurun_out/gab_gf$i.log 2>&1 && ms gpurun_out/gab_gf$i.log graph_nofwdproj || exit 1
done
