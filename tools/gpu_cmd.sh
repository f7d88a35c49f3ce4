ZT_LIB=$PWD/zlib.ts_amd/libzt_cnt.so timeout -k 10 300 python tools/df_count.py wordsalad structured xorshift32 2>&1 | grep -v amdgpu.ids
