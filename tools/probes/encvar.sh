set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
L=tyche_amd/libtyche_codec.so,tyche_amd/libtyche_codec_enc_wpe6.so,tyche_amd/libtyche_codec_enc_wpe6_lz4_hash_log9.so
TYCHE_LIBS=$L timeout -k 10 200 python tools/time_decode.py > gpurun_out/enc_h9.log 2>&1
for sp in "6144 22" "4096 22" "8192 22" "4096 0"; do set -- $sp; echo "seed $1 p0 $2" >> gpurun_out/enc_h9.log
 TYCHE_LZ4_ENC_SEED=$1 TYCHE_LZ4_ENC_P0=$2 TYCHE_LIBS=tyche_amd/libtyche_codec_enc_wpe6_lz4_hash_log9.so timeout -k 10 100 python tools/time_decode.py >> gpurun_out/enc_h9.log 2>&1; done
for a in "" "-w 2" "-w 4" "-U 80"; do ALL=1 WD=8 timeout -k 10 150 python tools/c1_fail_probe.py gpurun_out/c1fail2 6 $a >> gpurun_out/c1fail2.log 2>&1; done
