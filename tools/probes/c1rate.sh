export TMPDIR=/tmp
mkdir -p gpurun_out
for a in "-d 1" "-d 1 -m 256000" "-d 1 -m 1024000" "-d 1 -f 50" "-d 1 -w 2 -m 256000"; do ALL=1 WD=3 timeout -k 10 150 python tools/c1_fail_probe.py gpurun_out/c1fail3 12 $a >> gpurun_out/c1fail3.log 2>&1 || exit 1; done
