"""Summarise a wave timeline (SQ_TIMELINE=1 builds; bench.py writes it when
SQ_TIMELINE_OUT is set): per-wave start / stream-start / end in
s_memrealtime ticks (100 MHz).  Prints the launch span, per-wave phase
durations, and how many waves are resident / streaming over time, so that a
tail (the last waves running on a partly idle chip) can be told apart from a
slow steady state.
usage: python scripts/timeline.py tl.npy [bytes_per_launch]"""
import json
import sys

import numpy as np

tl = np.load(sys.argv[1]).astype(np.int64)
tl = tl[tl[:, 2] > 0]
t0 = tl[:, 0].min()
a, b, e = (tl[:, 0] - t0) * 10, (tl[:, 1] - t0) * 10, (tl[:, 2] - t0) * 10  # ns
span = e.max()
bins = np.arange(0, span + 1000, 1000)  # 1 us bins
alive = np.zeros(len(bins), np.int64)
strm = np.zeros(len(bins), np.int64)
ia, ib, ie = (np.searchsorted(bins, x) for x in (a, b, e))
np.add.at(alive, ia, 1)
np.add.at(alive, ie, -1)
np.add.at(strm, ib, 1)
np.add.at(strm, ie, -1)
alive, strm = np.cumsum(alive), np.cumsum(strm)
peak = np.percentile(alive, 90)
low = np.nonzero(alive >= 0.9 * peak)[0]
out = {
    "waves": int(len(tl)),
    "span_us": round(span / 1e3, 1),
    "prologue_us": [round(float(np.percentile(b - a, q)) / 1e3, 2) for q in (10, 50, 90)],
    "stream_us": [round(float(np.percentile(e - b, q)) / 1e3, 2) for q in (10, 50, 90)],
    "resident_peak": int(peak),
    "streaming_median": int(np.median(strm[: len(strm) * 9 // 10])),
    "ramp_us": round(float(low[0]), 1) if len(low) else None,
    "tail_us": round(float(span / 1e3 - low[-1]), 1) if len(low) else None,
    "first_end_us": round(float(e.min()) / 1e3, 1),
    "last_start_us": round(float(a.max()) / 1e3, 1),
}
if len(sys.argv) > 2:
    nbytes = float(sys.argv[2])
    # steady-state rate: bytes of waves that ran entirely inside [ramp, end of full occupancy]
    out["avg_TBps"] = round(nbytes / span / 1e3, 3)
print(json.dumps(out))
prof = [int(alive[i]) for i in range(0, len(alive), max(1, len(alive) // 40))]
print("resident waves every ~%d us:" % max(1, len(alive) // 40), prof)
