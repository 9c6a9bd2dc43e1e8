"""C2 (1024 x 1 MiB random) scan: would stopping a stream's later segments
after its first hit shorten the step?  A list-scheduling model of the scan's
work items (64 lanes x S bytes each, +64 warm-up bytes per lane) on the
chip's 4096 wave slots, in queue order (item j of every stream, then j + 1);
an item of a stream whose hit is already known (an earlier item found it) is
skipped, one running past it exits at its next poll.  Prints lane/ref and
the makespan against the no-skip schedule.

  python tools/c2_skip_model.py
"""
import numpy as np, heapq
MIN=512<<10; N=1<<20; R=N-MIN-64
rng=np.random.default_rng(1)
ns=1024; slots=4096
h=rng.exponential(1<<20, ns)  # first pure hit offset in the region
ref = np.minimum(h, R).sum()
for S in (256,512,1024,2048):
    ispan=64*S; ni=-(-R//ispan)
    # jobs in order item j for all streams
    jobs=[(j,s) for j in range(ni) for s in range(ns)]
    free=[0.0]*slots; heapq.heapify(free)
    found={}  # stream -> global time the hit becomes known
    lane=0
    # items of a stream in order; hit item k = h//ispan
    for j,s in jobs:
        t=heapq.heappop(free)
        hs=h[s]; hk=int(hs//ispan) if hs<R else 10**9
        if s in found and found[s]<=t and j>hk:
            heapq.heappush(free,t); continue
        dur=S+64
        end=t+dur
        if j>hk and s in found: end=min(end,max(t,found[s])+8)  # exits at the next poll
        if j==hk:
            tf=t+64+(hs%S)
            found[s]=min(found.get(s,1e18),tf)
        lane+= (end-t)*64
        heapq.heappush(free,end)
    mk=max(free)
    print(f"S={S} items/stream={ni} lane/ref={lane/ref:.3f} makespan={mk:.0f} (vs no-skip {(S+64)*ni*ns/slots:.0f})")
