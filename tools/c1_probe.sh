# builds the sample dir via pytest fixture path? simpler: use python to write sample pages
python - <<'PY'
import os, sys, hashlib
sys.path.insert(0, '.')
from tests.conftest import load_golden
from oracle import oracle as O
g = load_golden("lz4_sample.npz")
root = "/tmp/sd"
for i, name in enumerate(g["names"]):
    comp = g["comp"][g["comp_off"][i]:g["comp_off"][i] + g["comp_len"][i]]
    r, page = O.lz4_decompress(comp, int(g["size"][i]))
    path = os.path.join(root, str(name)); os.makedirs(os.path.dirname(path), exist_ok=True)
    open(path, "wb").write(page)
print("ok")
PY
for args in "-U 100" "-U 50" "" ; do
 for f in 0 2; do
  echo "=== args [$args] fail_every $f"
  TYCHE_APP_WATCHDOG=15 TYCHE_LOG_ERRORS=1 TYCHE_FAIL_COMPRESS_EVERY=$f timeout -k 5 40 integration/_app/tyche_q -c lz4 -p /tmp/sd/16k -w 1 -d 3 -m 512000 -f 20 $args > /tmp/o.txt 2> /tmp/e.txt
  echo "rc=$?"; grep -a "Compressions\|Restorations\|Updates\|Hits" /tmp/o.txt | head -5; echo "engine errors: $(grep -ac tyche-engine /tmp/e.txt)"; grep -a "fatal\|Comps" /tmp/e.txt | tail -2 | cut -c1-300; grep -a -A12 "fatal signal" /tmp/e.txt | head -14
 done
done
