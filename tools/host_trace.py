"""Summarise a JPGE_HOST_TRACE file: per encode_batch call the lane start/end
offsets, and for the slowest call each lane's iterations with the table jobs'
submit/start/done times (us, relative to the call's entry)."""
import sys


def load(fn):
    calls, lanes = [], []
    cur = []
    for line in open(fn):
        a, b, c, ln, x, y, z = line.split()
        a, b, ln = int(a), int(b), int(ln)
        if a == -2:
            calls.append((float(x), float(y), float(z)))
        elif a == -1:
            lanes.append((ln, float(x), float(y), cur))
            cur = []
        else:
            cur.append((a, b, float(c), float(x), float(y), float(z)))
    return sorted(calls), lanes


def main():
    calls, lanes = load(sys.argv[1])
    spans = sorted(((z - x, x, z) for x, y, z in calls[4:]), reverse=True)  # skip guard + warm-up
    d, x0, x1 = spans[0]
    print(f"slowest call {d:.0f} us (median {spans[len(spans) // 2][0]:.0f})")
    for ln, s, e, it in lanes:
        if s < x0 - 1 or e > x1 + 1:
            continue
        off = s - x0
        print(f" lane {ln}: start +{off:.0f} end +{e - x0:.0f}")
        for i, p, t, js, jst, jd in it:
            if p == 1 and js:
                print(f"   it {i:2d} tables ready at +{t + off:7.1f}; job submit +{js + off:7.1f} "
                      f"start +{jst + off:7.1f} done +{jd + off:7.1f}")
            if p == 4:
                print(f"   it {i:2d} finished drain at +{t + off:7.1f}")


if __name__ == "__main__":
    main()
