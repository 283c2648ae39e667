#!/bin/bash
# SQ counter passes (issue / stall mix) over one C2 bench step: per-kernel table.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/pmc_quick.sh gpurun_out/sq || { tail -5 gpurun_out/sq.p1.log gpurun_out/sq.p2.log; exit 1; }
python tools/pmc_table.py gpurun_out/sq/p1/p_counter_collection.csv gpurun_out/sq/p2/p_counter_collection.csv \
    > gpurun_out/sq_table.txt && grep -A17 -E "^k_(count_items|extract_scatter|part_scatter_tile|compact_items)" gpurun_out/sq_table.txt
