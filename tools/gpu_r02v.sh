set -euo pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r02v; mkdir -p $OUT
timeout -k 10 60 ./tools/ubench/l2_persist
cd /tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -T -f csv -d "$OUT/pmc" -o run -- $ROOT/tools/ubench/l2_persist > $OUT/pmc.log 2>&1
cd $ROOT
python3 - <<'P'
import csv
rows=list(csv.DictReader(open('gpurun_out/r02v/pmc/run_counter_collection.csv')))
rows.sort(key=lambda r:int(r['Dispatch_Id']))
vals=[float(r['Counter_Value']) for r in rows]
# per rep/shift: 20 iterations of (touch, reread); 3 reps x 2 shifts
i=0
for rep in range(3):
    for shift in range(2):
        rr=[vals[i+2*k+1] for k in range(20)]; tt=[vals[i+2*k] for k in range(20)]
        print('rep',rep,'shift',shift,'touch KiB median',sorted(tt)[10],'reread KiB median',sorted(rr)[10])
        i+=40
P
rm -f gpurun_out/r02v/pmc/run_counter_collection.csv
