#!/bin/bash
# Per-dispatch kernel trace + PMC counter passes for bench.py (run on the GPU box).
# usage: tools/prof_counters.sh OUTDIR [bench args...]
# One counter group per pass (rocprofv3 does not split passes; see MI355X_MICROARCH.md
# §rocprofv3 PMC slots): pmc1 instruction counts, pmc2 wait/busy cycles, pmc3 FETCH_SIZE,
# pmc4 WRITE_SIZE, pmc5 VALU issue cycles (SQ_ACTIVE_INST_VALU) with the launch's cycles,
# pmc6 the texture addresser's busy cycles (TA_BUSY_avr: per-XCD cycles the TA was busy).
# The PMC passes run one batch at a time on one stream (--overlap 0 --inflight 1: one
# dispatch per kernel per step, the launch structure of bench.py's one-stream pass); the
# trace runs the bench command as given.
set -e
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --cpu-seconds 0 --no-kernel-timing --serial-steps 0 "$@" > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $OUT/pmc1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 --no-kernel-timing --overlap 0 --inflight 1 "$@" > $OUT/pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d $OUT/pmc2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 --no-kernel-timing --overlap 0 --inflight 1 "$@" > $OUT/pmc2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc3 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 --no-kernel-timing --overlap 0 --inflight 1 "$@" > $OUT/pmc3.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d $OUT/pmc4 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 --no-kernel-timing --overlap 0 --inflight 1 "$@" > $OUT/pmc4.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d $OUT/pmc5 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 --no-kernel-timing --overlap 0 --inflight 1 "$@" > $OUT/pmc5.log 2>&1
timeout -k 10 300 rocprofv3 --pmc TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE -d $OUT/pmc6 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 --no-kernel-timing --overlap 0 --inflight 1 "$@" > $OUT/pmc6.log 2>&1
echo done
