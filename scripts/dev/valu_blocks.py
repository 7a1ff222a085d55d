"""Per-basic-block VALU / SALU / LDS / VMEM instruction counts of one kernel in a device .s file.

    hipcc ... --offload-device-only -S -o /tmp/wave.s hmc_wave.hip
    python scripts/dev/valu_blocks.py /tmp/wave.s 'k_wave_iters_k1ILb0ELb0ELb0ELb0ELb0E'

A static view for A/B work on instruction counts (the PMC SQ_INSTS_VALU pass is the measurement).
"""
import re
import sys


def kernel_lines(path, pat):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(pat) + r"\S*:", l))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    return lines[start:end + 1]


def main():
    path, pat = sys.argv[1], sys.argv[2]
    blocks, cur = [], ["entry", 0, 0, 0, 0, ""]
    for l in kernel_lines(path, pat):
        s = l.strip()
        m = re.match(r"^(\.LBB\S+):(.*)$", s) or re.match(r"^; %(bb\.\d+):(.*)$", s)
        if m:
            blocks.append(cur)
            cur = [m.group(1), 0, 0, 0, 0, m.group(2).strip()[:60]]
            continue
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        if op.startswith("v_"):
            cur[1] += 1
        elif op.startswith("s_") and op not in ("s_nop", "s_waitcnt"):
            cur[2] += 1
        elif op.startswith("ds_"):
            cur[3] += 1
        elif op.startswith(("global_", "buffer_", "scratch_")):
            cur[4] += 1
    blocks.append(cur)
    tot = [0, 0, 0, 0]
    print(f"{'block':14s} {'VALU':>5s} {'SALU':>5s} {'LDS':>4s} {'VMEM':>4s}  note")
    for b in blocks:
        print(f"{b[0]:14s} {b[1]:5d} {b[2]:5d} {b[3]:4d} {b[4]:4d}  {b[5]}")
        for i in range(4):
            tot[i] += b[i + 1]
    print(f"{'total':14s} {tot[0]:5d} {tot[1]:5d} {tot[2]:4d} {tot[3]:4d}")


if __name__ == "__main__":
    main()
