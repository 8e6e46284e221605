# round-4 last check (dev tool): smoke() and the row-block timings at the final head
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04.log 2>&1 || exit 1
tail -2 gpurun_out/smoke_r04.log
for P in 1 2; do timeout -k 10 240 python3 tools/dist_objective.py --loopback $P --points 16384 --dims 10 --grad --check || exit 1; done > gpurun_out/dist_r04final.log 2>&1
