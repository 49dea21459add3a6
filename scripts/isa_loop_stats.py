"""Instruction mix per basic block of one kernel in a hipcc -S listing.

    hipcc ... --cuda-device-only -S rsac_kernels.hip -o /tmp/k.s
    python scripts/isa_loop_stats.py /tmp/k.s <mangled-kernel-name> [min-instructions]

Prints, for every block with at least min-instructions instructions: VALU, SALU, LDS and other
(memory) instruction counts, and the number of lane ops (v_readlane / v_writelane: SGPR spills
show up here).
"""
import re
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    lim = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    s = open(path).read()
    i = s.index(name + ":")
    j = s.index(".Lfunc_end", i)
    cur, order, cnt = None, [], {}
    for line in s[i:j].split("\n"):
        line = line.strip()
        if re.match(r"^\.LBB\d+_\d+:", line):
            cur = line.split(":")[0]
            order.append(cur)
            cnt[cur] = [0, 0, 0, 0, 0]
        elif cur and line and not line.startswith((";", ".")):
            op = line.split()[0]
            k = 0 if op.startswith("v_") else 1 if op.startswith("s_") else 2 if op.startswith("ds_") else 3
            cnt[cur][k] += 1
            if "lane" in op:
                cnt[cur][4] += 1
    for o in order:
        c = cnt[o]
        if sum(c[:4]) >= lim:
            print(f"{o}: valu {c[0]} salu {c[1]} lds {c[2]} mem {c[3]} lane-ops {c[4]}")


if __name__ == "__main__":
    main()
