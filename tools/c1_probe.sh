# Diagnostic (GPU box): how the reference app behaves under an injected device failure, per caller
# variant, a few attempts each (the reference's list code is racy).  Writes the sample pages to /tmp/sd.
python - <<'PY'
import os, sys
sys.path.insert(0, '.')
from tests.conftest import load_golden
from oracle import oracle as O
g = load_golden("lz4_sample.npz")
for i, name in enumerate(g["names"]):
    comp = g["comp"][g["comp_off"][i]:g["comp_off"][i] + g["comp_len"][i]]
    r, page = O.lz4_decompress(comp, int(g["size"][i]))
    path = os.path.join("/tmp/sd", str(name)); os.makedirs(os.path.dirname(path), exist_ok=True)
    open(path, "wb").write(page)
PY
for app in ${APPS:-tyche_q tyche_fixed}; do
 for a in $(seq 1 ${RUNS:-3}); do
  echo "=== $app -U ${UPD:-50} fail_every ${FAIL:-2} attempt $a"
  TYCHE_APP_WATCHDOG=15 TYCHE_LOG_ERRORS=1 TYCHE_FAIL_COMPRESS_EVERY=${FAIL:-2} timeout -k 5 40 integration/_app/$app -c lz4 -p /tmp/sd/16k -w 1 -d 3 -m 512000 -f 20 -U ${UPD:-50} > /tmp/o.txt 2> /tmp/e.txt
  echo "rc=$?"; grep -a "Compressions\|Restorations\|Updates" /tmp/o.txt | head -3; echo "engine errors: $(grep -ac tyche-engine /tmp/e.txt)"
  grep -ao "[0-9.]*\S\? Comps ([0-9.]*\S\? Res)" /tmp/e.txt | tail -1; grep -a -A8 "fatal signal" /tmp/e.txt | grep -a "manager\|list\|buffer" | head -3
  [ -n "$VERBOSE" ] && grep -a -m1 -A25 "fatal signal" /tmp/e.txt | cut -c1-200; [ -n "$VERBOSE" ] && grep -a -m3 "tyche-engine" /tmp/e.txt
  grep -a -A30 "^--- thread" /tmp/e.txt | grep -ao "(\(list\|manager\|buffer\|tyche\)[a-z_]*" | sort | uniq -c | head -8
 done
done
