mkdir -p gpurun_out/anom
timeout -k 10 240 tools/debug/build/last_vgpr_ops 256 > gpurun_out/anom/last_vgpr_ops.txt 2>&1
echo rc=$?
