mkdir -p gpurun_out/band2
timeout -k 10 400 python -u tools/phase_band.py 10 > gpurun_out/band2/phase_band_r3q.txt 2>&1; rc=$?; grep -v "^{" gpurun_out/band2/phase_band_r3q.txt | tail -n 14; exit $rc
