#!/bin/bash
# Host issue rate vs GPU step time; eager vs segmented-graph A/B on one box
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/host_issue_probe.py > gpurun_out/r4_host.log 2>&1 && tail -1 gpurun_out/r4_host.log &&
for i in 1 2; do
timeout -k 10 200 python bench.py --graph 0 > gpurun_out/r4_ge$i.log 2>&1 && tail -1 gpurun_out/r4_ge$i.log | cut -c1-160 &&
timeout -k 10 200 python bench.py --graph 1 > gpurun_out/r4_gg$i.log 2>&1 && tail -1 gpurun_out/r4_gg$i.log | cut -c1-160 || exit 1
done
