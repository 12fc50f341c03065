"""Extract the stream operations a HIP-graph capture recorded from an AMD_LOG_LEVEL=3
AMD_LOG_MASK=1 log (the HIP runtime's API trace) and check them for what a capture cannot
express: waits on events never recorded inside the capture, streams forked into the capture
but never joined back into the origin stream. Writes the operations as a replay file for
tools/capture_repro (mode `file`).

    python tools/capture_ops.py gpurun_out/caplog.txt [out.ops]
"""
import re
import sys

ANSI = re.compile(r"\x1b\[[0-9;]*m")


def parse(path, pre=None):
    """(origin, priorities, captured ops); pre: a list that receives the operations logged before
    the capture began (the warm-up call on the same streams and events)."""
    prio = {}
    ops = []
    origin = None
    inside = False
    for line in open(path, errors="replace"):
        line = ANSI.sub("", line)
        m = re.search(r"hipStreamCreateWithPriority \( \S+, (\d+), (-?\d+) \)", line)
        if m:
            pend = int(m.group(2))
            continue
        m = re.search(r"hipStreamCreateWithPriority: Returned hipSuccess : stream:(\S+)", line)
        if m:
            prio[m.group(1)] = pend
            continue
        m = re.search(r"hipStreamBeginCapture \( stream:(\S+),", line)
        if m:
            origin, inside = m.group(1), True
            continue
        if not inside:
            if pre is not None:
                op = _op(line)
                if op:
                    pre.append(op)
            continue
        if "hipStreamEndCapture (" in line:
            break
        m = re.search(r"hipEventRecord \( event:(\S+), stream:(\S+) \)", line)
        if m:
            ops.append(("R", m.group(1), m.group(2)))
            continue
        m = re.search(r"hipStreamWaitEvent \( stream:(\S+), event:(\S+), (\d+) \)", line)
        if m:
            ops.append(("W", m.group(2), m.group(1)))
            continue
        m = re.search(r"hipLaunchKernel \( (\S+), \{(\d+),(\d+),(\d+)\}, \{(\d+),(\d+),(\d+)\}, \S+, "
                      r"(\d+), stream:(\S+) \)", line)
        if m:
            ops.append(("K", m.group(9), tuple(int(m.group(i)) for i in range(2, 9)), m.group(1)))
            continue
        m = re.search(r"(hipMemsetAsync|hipMemcpyAsync|hipMemcpyWithStream) \((.*)\)", line)
        if m:
            ops.append(("M", m.group(1), m.group(2)))
    return origin, prio, ops


def _op(line):
    m = re.search(r"hipEventRecord \( event:(\S+), stream:(\S+) \)", line)
    if m:
        return ("R", m.group(1), m.group(2))
    m = re.search(r"hipStreamWaitEvent \( stream:(\S+), event:(\S+), (\d+) \)", line)
    if m:
        return ("W", m.group(2), m.group(1))
    m = re.search(r"hipLaunchKernel \( (\S+), \{(\d+),(\d+),(\d+)\}, \{(\d+),(\d+),(\d+)\}, \S+, "
                  r"(\d+), stream:(\S+) \)", line)
    if m:
        return ("K", m.group(9), tuple(int(m.group(i)) for i in range(2, 9)), m.group(1))
    return None


def check(origin, ops):
    """Capture membership per stream (joined via a wait on an event recorded in the capture),
    waits on events not recorded in the capture, and streams whose last work is not ordered
    before the origin's last node."""
    recorded = {}   # event -> (stream, op index) of its latest record inside the capture
    member = {origin}
    issues = []
    for i, op in enumerate(ops):
        if op[0] == "R":
            if op[2] not in member:
                issues.append(f"op {i}: record on stream {op[2]} outside the capture")
            recorded[op[1]] = (op[2], i)
        elif op[0] == "W":
            if op[1] not in recorded:
                issues.append(f"op {i}: stream {op[2]} waits on event {op[1]} not recorded in "
                              f"the capture")
            member.add(op[2])
        elif op[0] == "K":
            if op[1] not in member:
                issues.append(f"op {i}: launch on stream {op[1]} outside the capture")
    # joined: the origin (transitively) waits on each member's last operation
    last = {}
    for i, op in enumerate(ops):
        st = op[2] if op[0] in ("R", "W") else op[1]
        last[st] = i
    # reachability: op j happens-before the origin's end if a chain of records/waits links them
    succ = {}
    prev_on = {}
    for i, op in enumerate(ops):
        st = op[2] if op[0] in ("R", "W") else op[1]
        if st in prev_on:
            succ.setdefault(prev_on[st], []).append(i)
        prev_on[st] = i
    rec_at = {}
    for i, op in enumerate(ops):
        if op[0] == "R":
            rec_at[op[1]] = i
        elif op[0] == "W" and op[1] in rec_at:
            succ.setdefault(rec_at[op[1]], []).append(i)
    end = last[origin]
    reach = {}

    def reaches(i):
        stack, seen = [i], set()
        while stack:
            j = stack.pop()
            if j == end:
                return True
            if j in seen:
                continue
            seen.add(j)
            stack.extend(succ.get(j, []))
        return False
    for st, i in last.items():
        if st != origin and not reaches(i):
            issues.append(f"stream {st}: its last op {i} ({ops[i][0]}) is not joined into the "
                          f"origin")
    return issues


def main():
    pre = []
    origin, prio, ops = parse(sys.argv[1], pre)
    streams = []
    for op in ops:
        st = op[2] if op[0] in ("R", "W") else op[1] if op[0] == "K" else None
        if st and st not in streams:
            streams.append(st)
    print(f"origin {origin}; {len(ops)} ops; streams (priority): "
          + ", ".join(f"{s}({prio.get(s, '?')})" for s in streams))
    kinds = {}
    for op in ops:
        kinds[op[0]] = kinds.get(op[0], 0) + 1
    print("ops:", kinds)
    for s in check(origin, ops):
        print("ISSUE", s)
    if len(sys.argv) > 2:
        sid = {s: i for i, s in enumerate([origin] + [s for s in streams if s != origin])}
        eid = {}
        with open(sys.argv[2], "w") as f:
            f.write(f"streams {len(sid)}\n")
            for s, i in sid.items():
                f.write(f"prio {i} {prio.get(s, 0)}\n")
            # the warm-up operations on the capture's streams (run before the capture begins)
            pre_ok = [op for op in pre if (op[2] if op[0] in ("R", "W") else op[1]) in sid]
            for op in pre_ok:
                if op[0] == "R":
                    f.write(f"r {eid.setdefault(op[1], len(eid))} {sid[op[2]]}\n")
                elif op[0] == "W":
                    f.write(f"w {eid.setdefault(op[1], len(eid))} {sid[op[2]]}\n")
                elif op[0] == "K":
                    g = op[2]
                    f.write(f"k {sid[op[1]]} {g[0]} {g[1]} {g[2]} {g[3]} {g[6]}\n")
            f.write("capture\n")
            for op in ops:
                if op[0] == "R":
                    f.write(f"R {eid.setdefault(op[1], len(eid))} {sid[op[2]]}\n")
                elif op[0] == "W":
                    f.write(f"W {eid.setdefault(op[1], len(eid))} {sid[op[2]]}\n")
                elif op[0] == "K":
                    g = op[2]
                    f.write(f"K {sid[op[1]]} {g[0]} {g[1]} {g[2]} {g[3]} {g[6]}\n")
        print(f"wrote {sys.argv[2]} ({len(eid)} events)")


if __name__ == "__main__":
    main()
