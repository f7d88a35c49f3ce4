for v in p2 cl16 cl4; do echo "== $v"; ZT_LIB=$PWD/zlib.ts_amd/build/var_$v/libzt.so timeout -k 10 300 python3 tools/df_digest.py wordsalad xorshift32 structured 2>&1 | grep L6; done
