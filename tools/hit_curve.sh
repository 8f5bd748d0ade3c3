set -e
cd tools
for n in 524288 131072; do
timeout -k 10 200 python seg_bench.py --n $n --hits 0,128,256,512,1024 2>&1 | grep -v amdgpu.ids | cut -c1-140
done
