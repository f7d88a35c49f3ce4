#!/bin/bash
# One parameterized GPU runner (round 6; replaces round 5's 47 one-off
# gpu_r05*.sh scripts, which git history keeps).  Runs the named steps in
# order on the GPU box, each under its own time limit, and stops at the first
# failing step.  Output goes to gpurun_out/TAG/.
#   usage: tools/gpu_run.sh TAG STEP [STEP ...]
# steps:
#   pytest            full -m gpu suite                       (pytest.log)
#   pytest:EXPR       -m gpu suite restricted by -k EXPR      (pytest.log)
#   smoke             __graft_entry__.smoke()                 (smoke.log)
#   bench             python bench.py (defaults)              (bench.log)
#   benchq            bench.py --steps 5 --no-cpu-baseline    (bench.log)
#   gate              16-window ratio gate                    (gate.log)
#   prof              rocprof kernel stats of 3 bench steps   (kernel_stats.csv)
#   c1 / c2 / c4      rocprof kernel stats of C1 / C2 / C4    (cN_kernel_stats.csv)
#   c4batch           C4 end to end                           (c4_batch.json)
#   c4host            C4 host stages on 8 aliased devices     (c4_host_stages.json)
#   api               host-API inflate time (appends)         (api.log)
#   apid              host-API deflate time (appends)         (apid.log)
#   infprof           rocprof kernel stats of infgen          (infgen_kernel_stats.csv)
#   infgen[:MiB]      foreign-stream inflate timing           (inflate_general_time.json)
#   infgenq           infgen, one summary line (appends)      (infgen.log)
#   kinds             per-generator deflate / inflate times   (kinds.log)
#   digest            stream digests (levels 6 / 1 / 9)       (digest.log)
#   node              Node facade bench (tools/node_bench.mjs) (node.log)
#   adapt:S1;S2;...   per-block depth sweep (ZT_DF_ADAPT settings) (adapt.log)
#   dftime            match-kernel cycle split (ab_dftime build)  (dftime.log)
#   regprobe          hipHostRegister vs pack of C4-sized buffers (regprobe.log)
#   lib=PATH          later steps load libzt from PATH (ZT_LIB); lib= resets
#   env=K=V           later steps see K=V; unenv=K removes K
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
ktimes() {  # kernel averages (ms) of a rocprof stats csv
  python3 - "$1" <<'EOF'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"  {r['Name'][:60]:60s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1e6:9.4f} ms")
EOF
}
prof() {  # prof NAME TIMEOUT -- cmd...
  local name=$1 to=$2; shift 3
  (cd /tmp && timeout -k 10 $to rocprofv3 --kernel-trace --stats -f csv -d $O/${name}_prof -o run -- "$@" > $O/${name}_prof.log 2>&1)
  cp $O/${name}_prof/run_kernel_stats.csv $O/${name}_kernel_stats.csv
  echo "$name kernel stats:"; ktimes $O/${name}_kernel_stats.csv | head -16
}
for step in "$@"; do
  echo "== $step"
  case $step in
    pytest) timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }; tail -1 $O/pytest.log ;;
    pytest:*) timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${step#pytest:}" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }; tail -1 $O/pytest.log ;;
    smoke) timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; tail -1 $O/smoke.log ;;
    bench) timeout -k 10 600 python3 bench.py > $O/bench.log 2>&1; tail -1 $O/bench.log ;;
    benchq) timeout -k 10 300 python3 bench.py --steps 5 --no-cpu-baseline > $O/bench.log 2>&1; tail -1 $O/bench.log ;;
    gate) timeout -k 10 300 python3 tools/ratio_gate.py > $O/gate.log 2>&1; tail -2 $O/gate.log ;;
    prof) prof bench 300 -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api --no-per-generator ;;
    c1) prof c1 180 -- python3 $R/tools/ck_time.py ;;
    c2) prof c2 300 -- python3 $R/tools/c2_bench.py 3 ;;
    c4) prof c4 300 -- python3 $R/tools/c4_batch.py 10000 ;;
    c4batch) timeout -k 10 300 python3 tools/c4_batch.py 10000 $O/c4_batch.json > $O/c4.log 2>&1; tail -3 $O/c4.log | cut -c1-300 ;;
    c4host) ZT_ALIAS_DEVICES=8 timeout -k 10 600 python3 tools/c4_host_stages.py 10000 $O/c4_host_stages.json > $O/c4_host_stages.log 2>&1; tail -5 $O/c4_host_stages.log ;;
    api) timeout -k 10 300 python3 tools/api_inflate_time.py >> $O/api.log 2>&1; echo "${ZT_LIB:-HEAD} $(tail -1 $O/api.log)" ;;
    apid) timeout -k 10 300 python3 tools/api_deflate_time.py >> $O/apid.log 2>&1; echo "${ZT_LIB:-HEAD} $(tail -1 $O/apid.log)" ;;
    infprof) prof infgen 600 -- python3 $R/tools/inflate_general_time.py 64 ;;
    infgen) timeout -k 10 600 python3 -u tools/inflate_general_time.py 64 $O/inflate_general_time.json > $O/infgen.log 2>&1; tail -1 $O/infgen.log | cut -c1-600 ;;
    infgenq) timeout -k 10 600 python3 -u tools/inflate_general_time.py 64 $O/inflate_general_time.json >> $O/infgen.log 2>&1; echo "$(env | grep ZT_GEN | tr '\n' ' ') $(tail -1 $O/infgen.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: (v["device"]["wall_ms"], v["device"]["passes_per_call"], v["host_api_GiBps"]) for k, v in d.items() if isinstance(v, dict)})')" ;;
    infgen:*) timeout -k 10 600 python3 -u tools/inflate_general_time.py ${step#infgen:} $O/inflate_general_time.json > $O/infgen.log 2>&1; tail -1 $O/infgen.log | cut -c1-600 ;;
    kinds) timeout -k 10 300 python3 tools/kind_time.py > $O/kinds.log 2>&1; tail -8 $O/kinds.log ;;
    digest) DF_LEVELS=6,1,9 timeout -k 10 300 python3 tools/df_digest.py wordsalad structured mixed > $O/digest.log 2>&1; grep -E 'L6|L1|L9' $O/digest.log ;;
    node) timeout -k 10 300 node --expose-gc tools/node_bench.mjs > $O/node.log 2>&1; tail -1 $O/node.log ;;
    adapt:*) IFS=';' read -ra A <<< "${step#adapt:}"; timeout -k 10 900 python3 -u tools/adapt_sweep.py "" "${A[@]}" > $O/adapt.log 2>&1; grep '^\[' $O/adapt.log ;;
    dftime) ZT_LIB=$R/zlib.ts_amd/build/ab_dftime/libzt.so timeout -k 10 300 python3 tools/df_time.py wordsalad structured > $O/dftime.log 2>&1; grep sub-chunk $O/dftime.log ;;
    regprobe) timeout -k 10 300 tools/micro/host_register_probe > $O/regprobe.log 2>&1; cat $O/regprobe.log ;;
    lib=) unset ZT_LIB ;;
    lib=*) export ZT_LIB=$R/${step#lib=} ;;
    env=*) export "${step#env=}" ;;
    unenv=*) unset "${step#unenv=}" ;;
    *) echo "gpu_run: unknown step $step" >&2; exit 2 ;;
  esac
done
