#!/bin/bash
O=gpurun_out/r03/ab_fused3
mkdir -p $O
TGSIM_LIB=$PWD/testground_amd/libtgsim_r02.so timeout -k 10 300 python scripts/stamps_chains.py > $O/stamps_r02_chains.log 2>&1 || { echo "stamps r02 failed"; tail $O/stamps_r02_chains.log; exit 1; }
head -14 $O/stamps_r02_chains.log
for v in "TGSIM_PRIO_HEAVY=0" "TGSIM_FUSED_WGS=2048" "TGSIM_PRIO_HEAVY=2048"; do
  env $v timeout -k 10 300 python scripts/stamps_chains.py > $O/stamps_$v.log 2>&1 || { echo "stamps $v failed"; tail $O/stamps_$v.log; exit 1; }
  echo "== $v"; head -6 $O/stamps_$v.log
done
timeout -k 10 300 python scripts/stamps.py --top 16 > $O/stamps_prof.log 2>&1 || { echo "stamps prof failed"; tail $O/stamps_prof.log; exit 1; }
cat $O/stamps_prof.log
