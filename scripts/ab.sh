#!/bin/bash
# A/B driver for one GPU call (replaces the ordinal one-shot drivers of rounds 3-5, which are in the
# git history).  For each variant, REPS interleaved bench lines (no CPU leg) of the given workloads,
# one summary line each.  A variant is "cur" (testground_amd/libtgsim.so), a library name
# (testground_amd/libtgsim_<name>.so, built by scripts/build_variant.sh) or ENV=VALUE pairs joined by
# commas (an engine knob on the current library).  Every GPU step has its own time limit; a failure
# stops the call.
#   VARIANTS="cur base TGSIM_FUSE=4" WORKLOADS="storm open epochs gossip" REPS=2 AB=name scripts/ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/ab/${AB:-ab}
mkdir -p "$out"
export TMPDIR=/tmp
stop() { echo "stopping after $1 (rc=$2)"; exit "$2"; }
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > "$out/pytest_gpu.log" 2>&1
  rc=$?; tail -2 "$out/pytest_gpu.log"; [ $rc -eq 0 ] || stop pytest $rc
fi
args_of() {  # bench arguments of a workload name
  case $1 in
    storm) echo "--no-1m --no-variants" ;;
    open) echo "--no-1m --no-variants --shapes open" ;;
    epochs) echo "--workload epochs" ;;
    gossip) echo "--workload gossip --peers 1000000" ;;
    gossip125k) echo "--workload gossip" ;;
    *) echo "$1" ;;
  esac
}
for rep in $(seq 1 "${REPS:-2}"); do
  for v in ${VARIANTS:-cur}; do
    lib=testground_amd/libtgsim.so; envs=()
    case $v in
      cur) ;;
      *=*) IFS=, read -ra envs <<< "$v" ;;
      *) lib=testground_amd/libtgsim_$v.so ;;
    esac
    for w in ${WORKLOADS:-storm}; do
      f="$out/${w}_${v//[=,\/]/_}_$rep.json"
      env "${envs[@]}" TGSIM_LIB="$PWD/$lib" timeout -k 10 300 python bench.py --no-cpu $(args_of "$w") ${BENCH_ARGS} \
        > "$f" 2> "${f%.json}.err" || stop "$w/$v" $?
      python - "$f" "$w" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[2]:10s} {sys.argv[3]:28s} {d['value'] / 1e9:8.3f} G pkt/s {d['ms_per_step']:.4f} ms/step "
      f"kernel {r['kernel_ms_avg']:.4f} ms carry {r['carry_bytes'] / 1e6:.1f} MB frac {r['frac']:.3f}")
PY
    done
  done
done
