"""CPU restatement of the device K8 stage — TEST INFRASTRUCTURE ONLY.

simple_reporter.py:176-187 filter + hour buckets, accumulated into the dense
[hour][segment][speed bin] count histogram that the HIP path reduces across GPUs."""
import math

import numpy as np

BINS = 8


def _py2_round_int(x):
    f = math.floor(x)
    return int(f + 1 if x - f >= 0.5 else f)


def histogram(res, first_time, last_time, seg_index_of_id, n_segments, base_time, hours, q=3600):
    """res: oracle/HIP result dict; first/last_time: per trace; seg_index_of_id: dict."""
    h = np.zeros((hours, n_segments, BINS), np.int64)
    rows = 0
    off = res['trace_rep_off']
    for t in range(len(off) - 1):
        buckets = (int(last_time[t]) - int(first_time[t])) // q + 1
        for k in range(off[t], off[t + 1]):
            t0, t1 = float(res['rep_t0'][k]), float(res['rep_t1'][k])
            ln, qu = int(res['rep_length'][k]), int(res['rep_queue'][k])
            if not (t0 > 0 and t1 > 0 and t1 - t0 > .5 and ln > 0 and qu >= 0):
                continue
            start, end = int(math.floor(t0)), int(math.ceil(t1))
            mn, mx = start // q, end // q
            if mx - mn > buckets:
                continue
            kmh = (ln / (t1 - t0)) * 3.6
            b = min(max(int(kmh / 20.0), 0), BINS - 1)
            seg = seg_index_of_id[int(res['rep_id'][k])]
            for bk in range(mn, mx + 1):
                rows += 1
                hh = (bk * q - base_time) // q
                if 0 <= hh < hours:
                    h[hh, seg, b] += 1
    return h, rows
