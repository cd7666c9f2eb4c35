#!/bin/bash
# Copy one GPU session's summaries (tools/session.sh TAG tests smoke bench counters workloads
# dropin) into profiles/.
# usage: [ROUND=r05] tools/collect_profiles.sh SESSION_TAG [PROFILE_TAG]
set -e
V=gpurun_out/$1
T=${2:-$1}
R=${ROUND:-r05}
cp $V/bench.json profiles/${R}_${T}_bench.json
[ -f $V/bench_inflight1.json ] && cp $V/bench_inflight1.json profiles/${R}_${T}_bench_inflight1.json
cp $V/prof/trace/run_kernel_stats.csv profiles/${R}_${T}_kernel_stats_b512.csv
cp $V/prof/pmc3/run_counter_collection.csv profiles/${R}_pmc_fetch_b512.csv
cp $V/prof/pmc4/run_counter_collection.csv profiles/${R}_pmc_write_b512.csv
cp $V/prof/pmc1/run_counter_collection.csv profiles/${R}_pmc_insts_b512.csv
cp $V/prof/pmc2/run_counter_collection.csv profiles/${R}_pmc_waits_b512.csv
cp $V/prof/pmc5/run_counter_collection.csv profiles/${R}_pmc_busy_b512.csv
[ -f $V/prof/pmc6/run_counter_collection.csv ] && cp $V/prof/pmc6/run_counter_collection.csv profiles/${R}_pmc_ta_b512.csv
[ -f $V/euroc.json ] && cp $V/euroc.json profiles/${R}_c3_euroc_bench.json
[ -f $V/reloc.json ] && cp $V/reloc.json profiles/${R}_c4_reloc_bench.json
[ -f $V/triangulation.json ] && cp $V/triangulation.json profiles/${R}_c5_triangulation_bench.json
[ -f $V/dropin.json ] && cp $V/dropin.json profiles/${R}_dropin_bench.json
[ -f $V/kfdb.json ] && cp $V/kfdb.json profiles/${R}_kfdb_bench.json
[ -f $V/tum.json ] && cp $V/tum.json profiles/${R}_c1_tum_bench.json
[ -f $V/bf.json ] && cp $V/bf.json profiles/${R}_c4_bf_bench.json
[ -f $V/hostio.json ] && cp $V/hostio.json profiles/${R}_hostio_graphs.json
[ -d $V/prof_euroc ] && cp $V/prof_euroc/trace/run_kernel_stats.csv profiles/${R}_euroc_kernel_stats_b256.csv
[ -d $V/prof_euroc ] && cp $V/prof_euroc/pmc3/run_counter_collection.csv profiles/${R}_pmc_fetch_euroc.csv
[ -d $V/prof_euroc ] && cp $V/prof_euroc/pmc4/run_counter_collection.csv profiles/${R}_pmc_write_euroc.csv
[ -d $V/prof_euroc ] && cp $V/prof_euroc/pmc1/run_counter_collection.csv profiles/${R}_pmc_insts_euroc.csv
[ -d $V/prof_euroc ] && cp $V/prof_euroc/pmc5/run_counter_collection.csv profiles/${R}_pmc_busy_euroc.csv
[ -f $V/prof_reloc/run_kernel_stats.csv ] && cp $V/prof_reloc/run_kernel_stats.csv profiles/${R}_c4_reloc_kernel_stats.csv
[ -f $V/prof_tri/run_kernel_stats.csv ] && cp $V/prof_tri/run_kernel_stats.csv profiles/${R}_c5_triangulation_kernel_stats.csv
for w in bf reloc triangulation; do
  [ -f $V/pmc_${w}_FETCH_SIZE.csv ] && cp $V/pmc_${w}_FETCH_SIZE.csv profiles/${R}_pmc_fetch_${w}.csv
  [ -f $V/pmc_${w}_WRITE_SIZE.csv ] && cp $V/pmc_${w}_WRITE_SIZE.csv profiles/${R}_pmc_write_${w}.csv
  [ -f $V/trace_${w}/run_kernel_stats.csv ] && cp $V/trace_${w}/run_kernel_stats.csv profiles/${R}_${w}_kernel_stats.csv
done
echo copied
