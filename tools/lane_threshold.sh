for n in 16384 32768 65536 131072; do
  for m in -1 0; do echo "pages=$n lane_min=$m"; PAGES=$n TYCHE_LZ4_LANE_MIN=$m timeout -k 10 120 python tools/time_decode.py 2>&1 | tail -1 || exit 1; done
done
