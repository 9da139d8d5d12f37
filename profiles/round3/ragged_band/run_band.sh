# ragged block kernel across group shapes, aligned (16) and packed (1) payloads
mkdir -p gpurun_out/band
B=tools/tune/build
for cfg in "5 11 64 1287" "5 11 64 400" "5 11 1000 351" "2 3 64 1287" "20 21 64 1287"; do
  for al in 16 1; do
    slot=1536; [ $al = 1 ] && slot=1452
    tag=$(echo "$cfg" | tr ' ' '_')_a$al
    TUNE_RW_PALIGN=$al TUNE_RW_BLOCKD=1 timeout -k 10 120 $B/tune_rw 10 3 $cfg 0 $slot > gpurun_out/band/$tag.txt 2>&1 || exit $?
    echo "== $cfg align $al"; tail -n 9 gpurun_out/band/$tag.txt | grep -E "product|nostore|multi2|groups"
  done
done
