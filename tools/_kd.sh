set -e
for s in 4096,262144,768 4096,262144,1536 4096,131072,3072 4096,65536,6144; do
  EBT_KB_THR=inf timeout -k 10 120 python tools/kernel_bench.py --one --shape $s 2>/dev/null | grep kernel
done
