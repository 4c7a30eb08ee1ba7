export PAGES=262144
echo "== wpe2 r192"; TYCHE_LIBS=tyche_amd/libtyche_codec.so python -u tools/time_decode.py
echo "== wpe2 r128"; TYCHE_LZ4_LC_RING=128 TYCHE_LIBS=tyche_amd/libtyche_codec.so python -u tools/time_decode.py
echo "== wpe3 r128"; TYCHE_LZ4_LC_RING=128 TYCHE_LIBS=tyche_amd/libtyche_codec_lc_wpe3.so python -u tools/time_decode.py
echo "== wpe3 r192"; TYCHE_LIBS=tyche_amd/libtyche_codec_lc_wpe3.so python -u tools/time_decode.py
