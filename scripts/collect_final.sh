#!/bin/bash
# Copy the judged outputs of scripts/gpu_final.sh (gpurun_out/${R}_*) into profiles/ as ${R}_final_*:
# bench lines, rocprofv3 kernel statistics, the pytest log and smoke, and the PMC record set.
set -u
cd "$(dirname "$0")/.."
R=${R:-r06}
for f in gpurun_out/${R}_pytest.log gpurun_out/${R}_smoke.log; do
  [ -f "$f" ] && cp "$f" "profiles/${R}_final_$(basename "$f" | sed "s/^${R}_//")"
done
for tag in c2 f1 app nee c4 c4nee c5 pmcsim8_c2 pmcsim8_c4 pmcsim8_c5; do
  [ -f gpurun_out/${R}_${tag}_bench.json ] && cp gpurun_out/${R}_${tag}_bench.json profiles/${R}_final_bench_${tag}.json
  [ -f gpurun_out/${R}_${tag}_rocprof/run_kernel_stats.csv ] && \
    cp gpurun_out/${R}_${tag}_rocprof/run_kernel_stats.csv profiles/${R}_final_${tag}_rocprof_kernel_stats.csv
done
[ -f gpurun_out/${R}_bench.json ] && cp gpurun_out/${R}_bench.json profiles/${R}_final_bench_default.json
for n in 2 4 8; do for c in c2 c4 c5; do
  [ -f gpurun_out/${R}_sim${n}_$c.json ] && cp gpurun_out/${R}_sim${n}_$c.json profiles/${R}_final_sim${n}_$c.json
done; done
# the PMC records: the last round profile of the call holds every record collected on the box
last=$(ls -t gpurun_out/${R}_*_pmc_r02.json 2>/dev/null | head -1)
[ -n "$last" ] && cp "$last" profiles/pmc_r02.json
ls profiles | grep "${R}_final" | wc -l
