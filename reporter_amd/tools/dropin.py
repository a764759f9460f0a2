"""The JSON drop-in path measured as its callers use it (bench.py's json_dropin leg and
tools/bench_json.py; workload infrastructure, the product never imports it).

Bodies are Batch.java's POST /report bodies (Batch.java:56-65: uuid, match_options with
mode and levels only, the points as Point.java:59-65 prints them; accuracy only when the
workload's traces carry one), so the configured
defaults decide the matching, as the deployed service's config does.  Two request sizes:
whole traces, and the streaming windows BatchingProcessor.java:26-29 reports on (at least
10 points, 60 s and 500 m: consecutive `window`-point pieces of each trace).  Callers:
  * one otr_report_batch C call with every body (a batching caller, FFM / ctypes);
  * `threads` caller threads each blocking on its own otr_report with the coalescer on
    (Kafka stream threads / HTTP server threads).
Every rate is probes/s over the wall time of the whole set, host scan and format included.
"""
import ctypes
import math
import threading
import time

MODES = ('auto', 'bicycle', 'pedestrian')


def bodies(tr, window=None):
    """Batch.java bodies of every trace (window=None) or of its consecutive window-point
    pieces (pieces shorter than 2 points dropped); returns (bodies as bytes, probes)."""
    out, probes = [], 0
    for t in range(tr.n_traces):
        a, b = int(tr.offsets[t]), int(tr.offsets[t + 1])
        cuts = [(a, b)] if not window else [(i, min(b, i + window)) for i in range(a, b, window)]
        mode = MODES[int(tr.mode[t])] if int(tr.mode[t]) < len(MODES) else 'auto'
        for i0, i1 in cuts:
            if i1 - i0 < 2:
                continue
            if tr.accuracy is None:
                pts = ','.join('{"lat":%.6f,"lon":%.6f,"time":%d}' % (tr.lat[i], tr.lon[i], tr.time[i])
                               for i in range(i0, i1))
            else:  # (Point.java:63-64 prints an integer accuracy)
                pts = ','.join('{"lat":%.6f,"lon":%.6f,"time":%d,"accuracy":%d}' % (
                    tr.lat[i], tr.lon[i], tr.time[i], int(math.ceil(tr.accuracy[i]))) for i in range(i0, i1))
            out.append(('{"uuid":"%s","match_options":{"mode":"%s","report_levels":[0,1],'
                        '"transition_levels":[0,1]},"trace":[%s]}' % (tr.uuids[t], mode, pts)).encode())
            probes += i1 - i0
    return out, probes


def batch_call(matcher, bs, reps=2):
    """One otr_report_batch with every body (best of reps): seconds, codes, MB out, split."""
    from .. import _lib
    L = _lib.lib()
    n = len(bs)
    arr = (ctypes.c_char_p * n)(*bs)
    lens = (ctypes.c_size_t * n)(*[len(b) for b in bs])
    codes = (ctypes.c_int32 * n)()
    outs = (ctypes.c_void_p * n)()
    olens = (ctypes.c_size_t * n)()
    best, split, out_mb = None, None, 0.0
    for _ in range(reps):
        _lib.service_stats(reset=True)
        t = time.perf_counter()
        L.otr_report_batch(matcher._h, n, arr, lens, -1, codes, outs, olens)
        dt = time.perf_counter() - t
        st = _lib.service_stats()
        out_mb = sum(olens[i] for i in range(n)) / 1e6
        for i in range(n):
            L.otr_free(outs[i])
        if best is None or dt < best:
            best, split = dt, st
    return best, [codes[i] for i in range(n)], out_mb, split


def coalesced(M, bs, threads, max_traces, wait_us):
    """`threads` callers, each looping over its share of the bodies with a blocking
    otr_report, the coalescer on: seconds, responses (code, body) in body order, split."""
    from .. import _lib
    got = [None] * len(bs)
    M.coalesce(max_traces, wait_us)
    _lib.service_stats(reset=True)

    def worker(k):
        mk = M.Matcher()
        for i in range(k, len(bs), threads):
            got[i] = mk.report_json(bs[i])
        mk.close()

    th = [threading.Thread(target=worker, args=(k,)) for k in range(threads)]
    t = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.perf_counter() - t
    st = _lib.service_stats()
    M.coalesce(0)
    return dt, got, st


def coalesced_native(config, bs, threads, max_traces, wait_us, timeout=300):
    """The same with native caller threads (reporter_amd/tools/loadgen, a child process
    with its own configure; no interpreter lock between the callers, as Java's stream
    threads): its JSON line (probes_per_s, identical, split), or None without the binary."""
    import json
    import os
    import subprocess
    import tempfile
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'loadgen')
    if not os.path.exists(exe):
        return None
    with tempfile.TemporaryDirectory() as d:
        cfg, body = os.path.join(d, 'config.json'), os.path.join(d, 'bodies.txt')
        with open(cfg, 'w') as f:
            json.dump(config, f)
        with open(body, 'wb') as f:
            f.write(b'\n'.join(bs) + b'\n')
        p = subprocess.run([exe, cfg, body, str(threads), str(max_traces), str(wait_us)], capture_output=True,
                           text=True, timeout=timeout)
    if p.returncode != 0:
        raise RuntimeError('loadgen failed (%d): %s' % (p.returncode, p.stderr[-2000:]))
    return json.loads(p.stdout.strip().splitlines()[-1])


def split_ms(st):
    """The host split of a service_stats dict in ms, plus calls / device batches."""
    return {'calls': int(st['calls']), 'device_batches': int(st['device_batches']),
            'scan_ms': round(1e3 * st['scan_s'], 2), 'soa_ms': round(1e3 * st['soa_s'], 2),
            'device_ms': round(1e3 * st['device_s'], 2), 'format_ms': round(1e3 * st['format_s'], 2),
            'total_ms': round(1e3 * st['total_s'], 2)}


def measure(M, matcher, tr, window=12, threads=(64, 256), max_traces=4096, wait_us=2000, config=None):
    """The json_dropin object of bench.py: whole-trace bodies through one batch call and
    coalesced callers, and BatchingProcessor-sized windows through coalesced callers.
    config (the configure dict): the coalesced callers are native threads in a child
    process (loadgen); without it, Python threads of this process (whose interpreter
    lock serialises the callers between their calls)."""
    res = {}
    import os
    if config is not None and not os.path.exists(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'loadgen')):
        config = None  # (no loadgen binary)

    def callers(bs, n, probes, want):
        if config is not None:
            r = coalesced_native(config, bs, n, max_traces, wait_us)
            return {'probes_per_s': r['probes_per_s'], 'seconds': r['seconds'], 'identical_to_batch': r['identical'],
                    'callers': 'native threads (loadgen)', 'split': r['split']}
        dt, got, st = coalesced(M, bs, n, max_traces, wait_us)
        return {'probes_per_s': round(probes / dt, 1), 'seconds': round(dt, 4), 'identical_to_batch': got == want,
                'callers': 'python threads', 'split': split_ms(st)}

    whole, probes = bodies(tr)
    mb = sum(len(b) for b in whole) / 1e6
    dt, codes, out_mb, st = batch_call(matcher, whole)
    res['whole_traces'] = {'bodies': len(whole), 'probes': probes, 'MB_in': round(mb, 1), 'MB_out': round(out_mb, 1),
                           'batch_c_call': {'probes_per_s': round(probes / dt, 1), 'seconds': round(dt, 4),
                                            'ok_200': sum(1 for c in codes if c == 200), 'split': split_ms(st)}}
    # the responses of the batch call are the reference for the coalesced ones
    want = matcher.report_json_batch(whole) if config is None else None
    for n in threads:
        res['whole_traces']['coalesced_%d_threads' % n] = callers(whole, n, probes, want)
    small, sprobes = bodies(tr, window)
    want = matcher.report_json_batch(small) if config is None else None
    res['streaming_windows'] = {'points_per_body': window, 'bodies': len(small), 'probes': sprobes}
    for n in threads:
        res['streaming_windows']['coalesced_%d_threads' % n] = callers(small, n, sprobes, want)
    dt, codes, _, st = batch_call(matcher, small)
    res['streaming_windows']['batch_c_call'] = {'probes_per_s': round(sprobes / dt, 1), 'seconds': round(dt, 4),
                                                'split': split_ms(st)}
    res['coalescer'] = {'max_traces': max_traces, 'max_wait_us': wait_us,
                        'dispatchers': int(__import__('os').environ.get('OTR_COALESCE_DISPATCHERS', '2'))}
    return res
