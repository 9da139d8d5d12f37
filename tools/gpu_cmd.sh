mkdir -p gpurun_out/rs6
timeout -k 10 300 tools/tune/build/tune_phase 5 3 > gpurun_out/rs6/tune_phase_rs6.txt 2>&1; rc=$?; tail -n 22 gpurun_out/rs6/tune_phase_rs6.txt; exit $rc
