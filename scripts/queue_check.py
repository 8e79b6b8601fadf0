"""Which hardware queue each stream's kernels ran on, from a rocprofv3 kernel trace:
    python scripts/queue_check.py <kernel_trace.csv>
Prints kernels per (Stream_Id, Queue_Id) and whether the two streams with the most fs2 kernels (the
main chain and the weight-gradient side stream) shared a queue (the round-3 DP1 regression)."""
import collections
import csv
import sys

cnt = collections.Counter()
own = collections.Counter()  # the framework's kernels (runtime blits excluded)
for r in csv.DictReader(open(sys.argv[1])):
    if r.get("Kind") == "KERNEL_DISPATCH":
        cnt[(r["Stream_Id"], r["Queue_Id"])] += 1
        if r["Kernel_Name"].startswith(("fs2::", "void fs2::")):
            own[r["Stream_Id"]] += 1
for (s, q), n in sorted(cnt.items()):
    print(f"stream {s:>3} queue {q:>3}: {n} kernels")
top = [s for s, _ in own.most_common(2)]
queues = {s: {q for (s2, q) in cnt if s2 == s} for s in top}
shared = len(top) == 2 and bool(queues[top[0]] & queues[top[1]])
print(f"main stream {top[0]} on queues {sorted(queues[top[0]])}, side stream "
      f"{top[1] if len(top) > 1 else '-'} on queues {sorted(queues[top[1]]) if len(top) > 1 else '-'}: "
      f"{'SHARED' if shared else 'separate'}")
