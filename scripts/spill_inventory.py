"""Per-loop spill inventory of a kernel's gfx950 assembly (hipcc --cuda-device-only -S output, one kernel).

    python3 scripts/spill_inventory.py kernel.s

Counts scratch stores/loads (VGPR spills), v_readlane/v_writelane (SGPR spills to VGPR lanes), global
loads/stores and VALU per loop, from LLVM's "in Loop: Header=... Depth=N" block annotations (each
loop's own blocks, not its nested loops). Record: profiles/r06_bvh_spill_inventory.txt."""
import re,sys,collections
lines=open(sys.argv[1]).read().split('\n')
cur=('-',0); hdr_depth={}
cnt=collections.defaultdict(lambda: collections.Counter())
i=0
for i,l in enumerate(lines):
    m=re.match(r'^(\.LBB\w+|; %bb\.\d+):\s*;\s*in Loop: Header=(BB\w+) Depth=(\d+)',l)
    if m: cur=(m.group(2),int(m.group(3))); continue
    m=re.match(r'^(\.LBB\w+):\s*;\s*(Parent Loop|=>)',l)
    if m:
        # header block: find the "This Inner Loop Header: Depth=N" line
        j=i
        while j<len(lines) and 'Inner Loop Header' not in lines[j]: j+=1
        d=int(re.search(r'Depth=(\d+)',lines[j]).group(1))
        cur=(m.group(1)[1:],d); continue
    m=re.match(r'^(\.LBB\w+|; %bb\.\d+):',l)
    if m and 'Loop' not in l: cur=('-',0); continue
    s=l.strip()
    if s.startswith('scratch_store'): cnt[cur]['spill_st']+=1
    elif s.startswith('scratch_load'): cnt[cur]['spill_ld']+=1
    elif s.startswith('v_readlane') or s.startswith('v_writelane'): cnt[cur]['sgpr_spill_lane']+=1
    elif s.startswith('global_store'): cnt[cur]['global_st']+=1
    elif s.startswith('global_load'): cnt[cur]['global_ld']+=1
    elif s.startswith('v_'): cnt[cur]['valu']+=1
depth_of={}
for (h,d),c in sorted(cnt.items(), key=lambda x:(x[0][1],x[0][0])):
    print(f"depth {d} header {h:10s} " + " ".join(f"{k}={v}" for k,v in sorted(c.items())))
