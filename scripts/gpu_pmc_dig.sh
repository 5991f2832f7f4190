set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/dig
export DBGPU_LIB=$PWD/databend_amd/libdbgpu_agg_exp.so
for v in 1 0; do
  rm -rf gpurun_out/dig/d$v
  DBG_X_PPDIG=$v timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/dig/d$v/write -o write --output-format csv -- python3 -u scripts/pmc_run.py --config 4 --steps 1 > gpurun_out/dig/d$v.log 2>&1 || { tail -5 gpurun_out/dig/d$v.log; exit 1; }
  DBG_X_PPDIG=$v timeout -k 10 200 python -u bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline --extra-configs none > gpurun_out/dig/b$v.json 2> gpurun_out/dig/b$v.err || exit 1
  python3 - <<PY
import csv,glob,json
from collections import defaultdict
f=glob.glob('gpurun_out/dig/d$v/write/**/*counter_collection.csv',recursive=True)[0]
disp={}
for r in csv.DictReader(open(f)):
    k=int(r['Dispatch_Id']); disp.setdefault(k,[r['Kernel_Name'],0.0]); disp[k][1]+=float(r['Counter_Value'])
order=sorted(disp); marks=[k for k in order if 'dbg_marker' in disp[k][0]]
by=defaultdict(float)
for k in order:
    if marks[-2]<k<marks[-1]: by[disp[k][0].split('(')[0][:50]]+=disp[k][1]*1024/1e9
d=json.loads(open('gpurun_out/dig/b$v.json').read().strip().splitlines()[-1])
print('dig=$v', round(d['ms_per_step'],2),'ms', {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()})
for k,v in sorted(by.items(), key=lambda x:-x[1])[:4]: print('   write GB', k, round(v,2))
PY
done
