#!/bin/bash
# A/B: pull grid cap (GOSSIP_PULL_GRID) on the C4 bench, one GPU.  Output: gpurun_out/grid_ab/*.json
# usage: tools/grid_ab.sh STEPS WARMUP GRID...
set -e
mkdir -p gpurun_out/grid_ab
K=$1; W=$2; shift 2
for g in "$@"; do
  GOSSIP_PULL_GRID=$g timeout -k 10 240 python bench.py --steps $K --warmup $W --no-cpu-baseline \
    > gpurun_out/grid_ab/grid_${g}_k$K.json 2> gpurun_out/grid_ab/grid_${g}_k$K.err
  echo "grid $g K=$K W=$W done"
done
