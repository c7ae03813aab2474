# host facts that bound the exact-order replay: THP mode, CPU model and caches
mkdir -p gpurun_out
{
echo "thp enabled: $(cat /sys/kernel/mm/transparent_hugepage/enabled 2>&1)"
echo "thp defrag: $(cat /sys/kernel/mm/transparent_hugepage/defrag 2>&1)"
grep -E "Hugepagesize|HugePages_Total|AnonHugePages" /proc/meminfo
lscpu | grep -E "Model name|Socket|Core|Thread|L1d|L2|L3|MHz|NUMA node"
} > gpurun_out/host_probe.txt 2>&1
ULG_EXACT_PROF=1 timeout -k 10 200 python -u scripts/probe_exact.py c3 > gpurun_out/exact_c3.log 2>&1 &
P=$!
sleep 25
grep -E "AnonHugePages|Rss" /proc/$P/smaps_rollup >> gpurun_out/host_probe.txt 2>&1 || true
wait $P
