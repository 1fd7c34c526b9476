"""Per-wave timeline of nn_search_kernel launches (library built with
-DORPCD_WAVETIME, run with ORPCD_WAVETIME=<file>):

    python tools/wavetime.py FILE [--every 10]

Per launch: running starts, splits, waves, span (first wave entry to last
exit), mean wave duration, average resident waves (sum of durations / span),
and when 50% / 90% / 99% of the waves had exited (fraction of the span).
"""
import sys

import numpy as np


def launches(path):
    raw = open(path, "rb").read()
    off = 0
    while off < len(raw):
        pass_, nact, S, n = np.frombuffer(raw, np.int32, 4, off)
        off += 16
        rec = np.frombuffer(raw, np.uint64, 3 * n, off).reshape(n, 3)
        off += 24 * n
        yield int(pass_), int(nact), int(S), rec


def main():
    path = sys.argv[1]
    every = int(sys.argv[sys.argv.index("--every") + 1]) if "--every" in sys.argv else 10
    tot_span = tot_busy = 0.0
    print(f"{'pass':>4} {'nact':>4} {'S':>3} {'waves':>6} {'span us':>8} {'wave us':>8} {'resident':>8} "
          f"{'t50':>5} {'t90':>5} {'t99':>5} {'q/wave':>6} {'max':>5} {'@':>5} {'lastin':>6} {'ideal':>5}")
    for k, (p, nact, S, r) in enumerate(launches(path)):
        if len(r) == 0:
            continue
        t0, t1 = r[:, 0].astype(np.int64), r[:, 1].astype(np.int64)
        base = t0.min()
        span = (t1.max() - base) * 0.01  # 100 MHz ticks -> us
        dur = (t1 - t0) * 0.01
        ends = np.sort(t1 - base) * 0.01
        q = (r[:, 2] & np.uint64(0xFFFFF)).astype(np.int64)
        tot_span += span
        tot_busy += dur.sum()
        if k % every == 0:
            f = [ends[int(x * (len(ends) - 1))] / span for x in (0.5, 0.9, 0.99)]
            # max: longest wave / span; @: its entry / span; lastin: last wave entry / span;
            # ideal: max(longest wave, sum of durations / 5120 slots) / span
            im = int(np.argmax(dur))
            ideal = max(dur.max(), dur.sum() / 5120) / span
            print(f"{p:4d} {nact:4d} {S:3d} {len(r):6d} {span:8.1f} {dur.mean():8.2f} {dur.sum() / span:8.0f} "
                  f"{f[0]:5.2f} {f[1]:5.2f} {f[2]:5.2f} {q.mean():6.2f} {dur.max() / span:5.2f} "
                  f"{(t0[im] - base) * 0.01 / span:5.2f} {(t0.max() - base) * 0.01 / span:6.2f} {ideal:5.2f}")
    print(f"all launches: span {tot_span:.0f} us, average resident waves {tot_busy / tot_span:.0f}")
    if "--dump" in sys.argv:  # every `every`-th launch's records, for offline scheduling studies
        keep = {f"l{k}": r for k, (p, nact, S, r) in enumerate(launches(path)) if k % every == 0 and len(r)}
        np.savez_compressed(sys.argv[sys.argv.index("--dump") + 1], **keep)


if __name__ == "__main__":
    main()
