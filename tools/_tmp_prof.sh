export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29551
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/tl -o run -- python bench.py --force-shard --workload hier_fedbuff --hier-mode sync --steps 5 --warmup 2 --cpu-clients 0 > gpurun_out/tl_sync.log 2>&1
python - <<'PY'
import csv, glob
rows=[]
for f in glob.glob("gpurun_out/tl/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60], r.get("Stream_Id","?")))
for f in glob.glob("gpurun_out/tl/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY "+r.get("Direction","")+" "+r.get("Size",""), "copy"))
rows.sort()
# last 200 events after the first hier kernel of the timed region
hk=[i for i,r in enumerate(rows) if "hier" in r[2]]
start=hk[max(0,len(hk)-18)]
t0=rows[start][0]
with open("gpurun_out/tl_summary.txt","w") as o:
    prev=None
    for s,e,n,st in rows[start:]:
        o.write(f"{(s-t0)/1e3:10.1f} {(e-s)/1e3:9.1f} us  gap {((s-prev)/1e3 if prev else 0):9.1f}  {st}  {n}\n")
        prev=e
PY
rm -rf gpurun_out/tl
