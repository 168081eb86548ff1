#!/bin/bash
# A/B: product build vs the single-chain column-sum asm (BN_DOT2_ASM=1), configs 2, 5, 3 and G2*Fr
set -e
OUT=gpurun_out/r5b
mkdir -p $OUT
export TMPDIR=/tmp
BN254MI_LIB=ab/lib_asm.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "throughput or kat or config or product" > $OUT/asm_parity.log 2>&1 || { tail -30 $OUT/asm_parity.log; exit 1; }
tail -1 $OUT/asm_parity.log
timeout -k 10 900 bash tools/gpu_ab.sh r5b paritytech-bn_amd/libbn254mi.so ab/lib_asm.so "pairing product g2mul g1mul"
for f in $OUT/*_B_*.json $OUT/*_A_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d.get('parity_sample_bit_exact', d.get('parity_bit_exact')), d.get('roofline',{}).get('frac'))"; done
