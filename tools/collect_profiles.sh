#!/bin/bash
# Copy one GPU session's summaries (tools/gpu_session.sh TAG) into profiles/.
# usage: tools/collect_profiles.sh TAG
set -e
V=gpurun_out/$1
cp $V/bench.json profiles/r01_$1_bench.json
cp $V/prof/trace/run_kernel_stats.csv profiles/r01_$1_kernel_stats_b512.csv
cp $V/prof/pmc3/run_counter_collection.csv profiles/r01_pmc_fetch_b512.csv
cp $V/prof/pmc4/run_counter_collection.csv profiles/r01_pmc_write_b512.csv
cp $V/prof/pmc1/run_counter_collection.csv profiles/r01_pmc_insts_b512.csv
cp $V/prof/pmc2/run_counter_collection.csv profiles/r01_pmc_waits_b512.csv
cp $V/euroc.json profiles/r01_c3_euroc_bench.json
cp $V/reloc.json profiles/r01_c4_reloc_bench.json
cp $V/tri.json profiles/r01_c5_triangulation_bench.json
cp $V/prof_euroc/trace/run_kernel_stats.csv profiles/r01_euroc_kernel_stats_b256.csv
cp $V/prof_euroc/pmc3/run_counter_collection.csv profiles/r01_pmc_fetch_euroc.csv
cp $V/prof_euroc/pmc4/run_counter_collection.csv profiles/r01_pmc_write_euroc.csv
cp $V/prof_euroc/pmc1/run_counter_collection.csv profiles/r01_pmc_insts_euroc.csv
[ -f $V/prof_reloc/run_kernel_stats.csv ] && cp $V/prof_reloc/run_kernel_stats.csv profiles/r01_c4_reloc_kernel_stats.csv
[ -f $V/prof_tri/run_kernel_stats.csv ] && cp $V/prof_tri/run_kernel_stats.csv profiles/r01_c5_triangulation_kernel_stats.csv
ls $V/prof_reloc $V/prof_tri 2>/dev/null | head
echo copied
