# PMC HBM traffic of the current tree for C2 and C4 (tools/pmc_traffic.sh, one run each), then the C2 / C4 bench
# lines that attach them; outputs under gpurun_out/pmcfinal (copy the json into profiles/ to commit)
set -o pipefail
mkdir -p gpurun_out/pmcfinal
rm -rf gpurun_out/pmc_traffic
timeout -k 10 500 bash tools/pmc_traffic.sh r5_pmc_traffic_c2_f16_b32 --no-secondary > gpurun_out/pmcfinal/c2_pmc.log 2>&1 || { echo "c2 pmc failed"; tail -5 gpurun_out/pmcfinal/c2_pmc.log; exit 1; }
cp gpurun_out/pmc_traffic/r5_pmc_traffic_c2_f16_b32.json gpurun_out/pmcfinal/
rm -rf gpurun_out/pmc_traffic/p1 gpurun_out/pmc_traffic/p2
timeout -k 10 500 bash tools/pmc_traffic.sh r5_pmc_traffic_c4_f16_b8 --config c4 > gpurun_out/pmcfinal/c4_pmc.log 2>&1 || { echo "c4 pmc failed"; tail -5 gpurun_out/pmcfinal/c4_pmc.log; exit 1; }
cp gpurun_out/pmc_traffic/r5_pmc_traffic_c4_f16_b8.json gpurun_out/pmcfinal/
rm -rf gpurun_out/pmc_traffic/p1 gpurun_out/pmc_traffic/p2
echo "pmc done"
