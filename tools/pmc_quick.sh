set -e
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $OUT/pmc1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 --no-kernel-timing > $OUT/pmc1.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d $OUT/pmc2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 --no-kernel-timing > $OUT/pmc2.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM -d $OUT/pmc5 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 --no-kernel-timing > $OUT/pmc5.log 2>&1
echo pmc done
