set -e
mkdir -p gpurun_out/p1
ZT_LIB=$GRAFT_REPO_ROOT/zlib.ts_amd/build/var_time/libzt.so timeout -k 10 180 python3 -u tools/df_time.py wordsalad xorshift32 structured > gpurun_out/p1/time.log 2>&1
cat gpurun_out/p1/time.log
