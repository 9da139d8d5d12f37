mkdir -p gpurun_out
bash tools/pmc_protect.sh r2c > gpurun_out/pmc_protect_r2c.log 2>&1
echo rc=$?
