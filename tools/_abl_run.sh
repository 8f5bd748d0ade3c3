# GEMM ablation sweep: store/filter TFLOP/s of each _abl/libebert_<v>.so at the C3 chunk shape
set -e
for v in ${VARIANTS:-base noepi nowait sleep0 prio1 prio2 base}; do
  echo "$v $(EBT_KB_THR=inf EBERT_LIB=_abl/libebert_$v.so timeout -k 10 120 python tools/kernel_bench.py --one 2>/dev/null)"
done
cd tools && timeout -k 10 120 python blas_ref.py
