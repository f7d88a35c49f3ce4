#!/bin/bash
# chain-cut threshold / depth sweep on wordsalad and structured (level-6 base 32,128,1,128,8,16,16,1)
for p in 32,128,1,128,8,16,16,1 32,128,1,128,8,16,8,1 32,128,1,128,8,16,12,1 24,128,1,128,8,16,16,1 40,128,1,128,8,16,24,1 32,128,1,128,8,8,16,1; do
  for k in wordsalad structured; do
    timeout -k 10 120 python3 tools/df_sweep.py $k $p 2>&1 | grep ratio || exit 1
  done
done
