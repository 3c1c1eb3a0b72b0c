"""Per-kernel timeline of a few timed steps from a rocprofv3 kernel trace
(development aid; how profiles/r06m_fed_trace.txt .. r06o were made):
    python3 tools/fed_trace.py <kernel_trace.csv> <first step> <last step>
Steps count the last 20 k_motion dispatches before the final k_clock probe
(the timed region); each line: start, end, duration (us from the first
shown), hardware queue, kernel."""
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
idx=[i for i,r in enumerate(rows) if 'k_clock' in r['Kernel_Name']]
end=idx[-1]
km=[i for i in range(end) if 'k_motion' in rows[i]['Kernel_Name']][-20:]
t0=int(rows[km[0]]['Start_Timestamp'])
a,b=int(sys.argv[2]),int(sys.argv[3])
for i in range(km[a]-4, km[b]):
    r=rows[i]; s=int(r['Start_Timestamp'])-t0; e=int(r['End_Timestamp'])-t0
    print(f"{s/1e3:9.1f} {e/1e3:9.1f} {(e-s)/1e3:7.1f} q{r.get('Queue_Id','?')} {r['Kernel_Name'][:60]}")
