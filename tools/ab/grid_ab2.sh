#!/bin/bash
# A/B: pull grid cap on C3 (1M nodes) and on the N=8 per-rank share of C4.  Output: gpurun_out/grid_ab2/
set -e
mkdir -p gpurun_out/grid_ab2
for g in "$@"; do
  GOSSIP_PULL_GRID=$g timeout -k 10 200 python bench.py --workload C3 --no-cpu-baseline \
    > gpurun_out/grid_ab2/c3_$g.json 2> gpurun_out/grid_ab2/c3_$g.err
  GOSSIP_PULL_GRID=$g timeout -k 10 200 python bench.py --rehearse-shards 8 --no-cpu-baseline \
    > gpurun_out/grid_ab2/c4r8_$g.json 2> gpurun_out/grid_ab2/c4r8_$g.err
  echo "grid $g done"
done
