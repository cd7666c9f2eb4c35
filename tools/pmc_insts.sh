#!/bin/bash
# Instruction-mix counters per kernel for one bench step (run on the GPU box).
# usage: tools/pmc_insts.sh OUTDIR [bench args...]
set -e
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $OUT/pmc1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 --no-kernel-timing "$@" > $OUT/pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS -d $OUT/pmc2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 --no-kernel-timing "$@" > $OUT/pmc2.log 2>&1
python3 tools/pmc_summary.py $OUT/pmc1/*counter_collection.csv $OUT/pmc2/*counter_collection.csv
