#!/usr/bin/env python
"""Map the frames of a glog-style crash trace onto libraries (measurement aid, round 4).

    python tools/symbolize.py CRASH_LOG MAPS_FILE

The crashed process left no memory map, so its libraries are placed with the layout of a
probe run under the same launcher (tools/maps_probe.py writes its /proc/self/maps):
libraries mapped at start-up (LD_PRELOADs, their dependencies, libc) keep their distances, so
every frame near libc is shifted by (probe libc base - crash libc base), with the crash's libc
base taken from the signal trampoline frame (``__restore_rt``, found in this image's libc by
its ``mov $0xf,%rax; syscall`` bytes).  Prints library + offset per frame; the offsets are then
read with objdump against the same image's files (the ROCm libraries are stripped, so the
functions are identified from the instructions at those offsets).
"""
from __future__ import annotations

import re
import subprocess
import sys

LIBC = "/usr/lib/x86_64-linux-gnu/libc.so.6"


def restore_rt_offset() -> int:
    out = subprocess.run(["objdump", "-d", "--no-show-raw-insn", LIBC], capture_output=True, text=True).stdout
    lines = out.splitlines()
    for i, l in enumerate(lines[:-1]):
        if "mov    $0xf,%rax" in l and "syscall" in lines[i + 1]:
            return int(l.split(":")[0], 16)
    raise RuntimeError("no rt_sigreturn trampoline in libc")


def load_maps(path):
    regions = []
    for l in open(path):
        if l.startswith("#"):
            continue
        p = l.split()
        if len(p) >= 6 and p[5].startswith("/"):
            a, b = (int(x, 16) for x in p[0].split("-"))
            regions.append((a, b, p[5]))
    bases = {}
    for a, _b, name in regions:
        bases[name] = min(a, bases.get(name, a))
    return regions, bases


def main():
    log, maps = sys.argv[1], sys.argv[2]
    frames = [int(m.group(1), 16) for m in re.finditer(r"@\s+(0x[0-9a-f]+)", open(log).read())]
    pc = re.search(r"PC: @\s+(0x[0-9a-f]+)", open(log).read())
    if pc:
        frames.insert(0, int(pc.group(1), 16))
    regions, bases = load_maps(maps)
    libc_probe = next(v for k, v in bases.items() if k.endswith("/libc.so.6"))
    rr = restore_rt_offset()
    tramp = [f for f in frames if (f - rr) & 0xFFF == 0]
    if not tramp:
        raise SystemExit("no __restore_rt frame in the trace")
    shift = libc_probe - (tramp[0] - rr)
    print(f"crash libc base {tramp[0] - rr:#x} (frame {tramp[0]:#x} = __restore_rt + 0), probe libc base {libc_probe:#x}")
    for f in frames:
        g = f + shift
        hit = next(((a, b, n) for a, b, n in regions if a <= g < b), None)
        if hit:
            print(f"{f:#x}  {hit[2]} + {g - bases[hit[2]]:#x}")
        else:
            print(f"{f:#x}  (not in a start-up library of the probe layout)")


if __name__ == "__main__":
    main()
