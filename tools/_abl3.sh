cd tools
for rep in 1 2; do
for v in old sync new; do
  if [ $v = new ]; then L=$GRAFT_REPO_ROOT/robot_ebert_amd/libebert.so; else L=$GRAFT_REPO_ROOT/_abl/libebert_$v.so; fi
  for n in 524288 131072; do
    echo "$v n=$n $(EBERT_LIB=$L timeout -k 10 120 python seg_bench.py --n $n --hits 0,128,1024 --no-inf 2>/dev/null | python3 -c '
import sys,json
out=[]
for l in sys.stdin:
    d=json.loads(l)
    if "hits" in d: out.append("%s:%.4f" % (round(d["hits"]), d["ms"]))
print(" ".join(out))')"
  done
done
done
