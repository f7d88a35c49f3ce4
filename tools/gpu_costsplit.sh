set -e
timeout -k 10 300 python3 tools/ratio_gate.py "" "32,128,1,128,8,0,16,1" "32,128,1,128,8,8,16,1" "8,128,1,128,8,16,16,1" "1,128,1,128,8,16,16,1" > gpurun_out/nc_base.log 2>&1
ZT_LIB=$PWD/zlib.ts_amd/build/exp_nop4/libzt.so timeout -k 10 300 python3 tools/ratio_gate.py "" > gpurun_out/nc_nop4.log 2>&1
grep -h '^\[' gpurun_out/nc_base.log gpurun_out/nc_nop4.log
