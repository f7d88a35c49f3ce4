set -e
R=$PWD
for v in base b4t256 b4t512 b4t1024 b2t1024; do
  lib=$R/zlib.ts_amd/libzt.so; [ $v = base ] || lib=$R/zlib.ts_amd/build/var_$v/libzt.so
  ZT_LIB=$lib timeout -k 10 120 python3 tools/ck_check.py 2>&1 | grep -v amdgpu.ids
done
