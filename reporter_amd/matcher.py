"""Host-side handle over libotr: configuration and the batched matching API.

Mirrors the reference's process model: `configure()` once per process
(valhalla.Configure, reporter_service.py:284), one `Matcher` per thread
(reporter_service.py:51-52).
"""
import ctypes
import json
import os
import tempfile

import numpy as np

from . import _lib

P = ctypes.POINTER

MODES = {'auto': 0, 'bicycle': 1, 'pedestrian': 2}


OTR_KEYS = ('speed_kph', 'queue_kph', 'delta')  # engine keys, not meili's


def default_config(graph_path, device=0, **options):
    """Valhalla-style config dict of the reference deployment: valhalla_build_config's meili
    section (per-mode turn_penalty_factor auto 200 / bicycle 140 / pedestrian 100) with the
    Dockerfile's overrides (sigma_z 4.07, beta 3, max_route_distance_factor 5,
    max_route_time_factor 2; Dockerfile:14-17,42-49).  `options` apply to every mode, as a
    request's match_options override the configured values (generate_test_trace.py:44-52
    sends turn_penalty_factor 0, for example); speed_kph / queue_kph go to the otr section."""
    d = {'sigma_z': 4.07, 'beta': 3, 'max_route_distance_factor': 5, 'max_route_time_factor': 2,
         'breakage_distance': 2000, 'interpolation_distance': 10, 'search_radius': 50,
         'max_search_radius': 100, 'gps_accuracy': 5.0, 'turn_penalty_factor': 0, 'max_candidates': 32}
    modes = {'auto': {'turn_penalty_factor': 200, 'search_radius': 50},
             'bicycle': {'turn_penalty_factor': 140},
             'pedestrian': {'turn_penalty_factor': 100, 'search_radius': 50}}
    otr = {'graph': os.path.abspath(graph_path), 'device': device}
    for k, v in options.items():
        if k in OTR_KEYS:
            otr[k] = v
        else:
            d[k] = v
            for m in modes.values():
                m[k] = v
    return {'meili': dict(default=d, **modes), 'otr': otr}


def configure(config):
    """Configure from a path or a dict; raises RuntimeError on failure."""
    L = _lib.lib()
    if isinstance(config, dict):
        s = json.dumps(config).encode()
        rc = L.otr_configure_json(s, len(s))
    else:
        rc = L.otr_configure(os.fspath(config).encode())
    if rc != 0:
        raise RuntimeError('otr_configure failed (%d): %s' % (rc, _lib.last_error()))


def coalesce(max_traces, max_wait_us=2000):
    """Coalesce concurrent report_json calls of all threads into shared device batches
    (otr_coalesce); max_traces <= 0 stops it."""
    rc = _lib.lib().otr_coalesce(int(max_traces), int(max_wait_us))
    if rc != 0:
        raise RuntimeError('otr_coalesce failed (%d): %s' % (rc, _lib.last_error()))


def graph_info():
    a, b, c = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    rc = _lib.lib().otr_graph_info(ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
    if rc != 0:
        raise RuntimeError('not configured')
    return a.value, b.value, c.value


class IngestedBatch:
    """The traces otr_ingest left in HBM, in the shape match_batch takes."""

    def __init__(self, r):
        b = r.batch
        self.n_traces = int(r.n_traces)
        self.n_probes = int(r.n_probes)
        self.arrays = {'trace_offsets': b.trace_offsets, 'lat': b.lat, 'lon': b.lon, 'time': b.time,
                       'accuracy': b.accuracy, 'mode': b.mode}
        self.uuid_off = r.d_trace_uuid_off
        self.uuid_len = r.d_trace_uuid_len


class Matcher:
    def __init__(self):
        self._L = _lib.lib()
        self._h = self._L.otr_matcher_new()
        self._keep = []

    def close(self):
        if self._h:
            self._L.otr_matcher_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self):
        return self._L.otr_matcher_stream(self._h)

    # --- JSON drop-in entry points ------------------------------------------------
    def match_json(self, trace_json):
        """SegmentMatcher.Match(json) -> str (reporter_service.py:240)."""
        s = trace_json.encode() if isinstance(trace_json, str) else trace_json
        out, n = ctypes.c_void_p(), ctypes.c_size_t()
        rc = self._L.otr_match(self._h, s, len(s), ctypes.byref(out), ctypes.byref(n))
        body = _lib.take_string(out, n)
        if rc != 0:
            raise RuntimeError(json.loads(body).get('error', body) if body else _lib.last_error())
        return body

    def report_json(self, trace_json, threshold_sec=-1):
        """POST /report: returns (http_code, body) exactly as handle_request (209-245)."""
        s = trace_json.encode() if isinstance(trace_json, str) else trace_json
        out, n = ctypes.c_void_p(), ctypes.c_size_t()
        rc = self._L.otr_report(self._h, s, len(s), threshold_sec, ctypes.byref(out), ctypes.byref(n))
        return rc, _lib.take_string(out, n)

    def report_json_batch(self, bodies, threshold_sec=-1):
        """Many POST /report bodies in shared device batches (otr_report_batch):
        [(http_code, body)], item i exactly as report_json(bodies[i])."""
        enc = [b.encode() if isinstance(b, str) else bytes(b) for b in bodies]
        n = len(enc)
        arr = (ctypes.c_char_p * max(n, 1))(*enc)
        lens = (ctypes.c_size_t * max(n, 1))(*[len(b) for b in enc])
        codes = (ctypes.c_int32 * max(n, 1))()
        outs = (ctypes.c_void_p * max(n, 1))()
        olens = (ctypes.c_size_t * max(n, 1))()
        rc = self._L.otr_report_batch(self._h, n, arr, lens, threshold_sec, codes, outs, olens)
        if rc != 0:
            raise RuntimeError('otr_report_batch failed (%d): %s' % (rc, _lib.last_error()))
        res = []
        for i in range(n):
            res.append((codes[i], _lib.take_string(ctypes.c_void_p(outs[i]), ctypes.c_size_t(olens[i]))))
        return res

    # --- batched API ----------------------------------------------------------------
    def match_batch(self, traces, report_levels=(0, 1), transition_levels=(0, 1), threshold_sec=15,
                    quantisation=3600, hist_base_time=0, hist_hours=0, copy_out=True, timing=False,
                    device_arrays=None, hist_device=None, tile_rows=False, tile_rules=0, host_arrays=None,
                    copy_reports=False, route_work=False):
        """Match a gen.Traces-like SoA batch.  With device_arrays (dict of device
        pointers: trace_offsets, lat, lon, time, accuracy, mode) the inputs are
        already resident in HBM; host_arrays: the same as host pointers (e.g. pinned
        buffers the caller keeps alive).  copy_reports: segments, reports and stats
        come back to the host (the JSON path's copy-out).  route_work: the LDS route
        tiers count their work (route_tier_work; instrumentation, ~7% of the first tier)."""
        b = _lib.TraceBatch()
        b.n_traces = int(traces.n_traces)
        arrs = device_arrays if device_arrays is not None else host_arrays
        if arrs is not None:
            b.memory = _lib.OTR_MEM_DEVICE if device_arrays is not None else _lib.OTR_MEM_HOST
            b.trace_offsets = arrs['trace_offsets']
            b.lat = arrs['lat']
            b.lon = arrs['lon']
            b.time = arrs['time']
            b.accuracy = arrs.get('accuracy') or None
            b.mode = arrs['mode']
        else:
            b.memory = _lib.OTR_MEM_HOST
            keep = [np.ascontiguousarray(traces.offsets, np.int64), np.ascontiguousarray(traces.lat, np.float64),
                    np.ascontiguousarray(traces.lon, np.float64), np.ascontiguousarray(traces.time, np.int64),
                    np.ascontiguousarray(traces.mode, np.uint8)]
            acc = None if traces.accuracy is None else np.ascontiguousarray(traces.accuracy, np.float32)
            self._keep = keep + [acc]
            b.trace_offsets, b.lat, b.lon, b.time, b.mode = [k.ctypes.data for k in keep]
            b.accuracy = acc.ctypes.data if acc is not None else None
        b.report_levels = _lib.levels_mask(report_levels)
        b.transition_levels = _lib.levels_mask(transition_levels)
        b.threshold_sec = threshold_sec
        b.quantisation = quantisation
        b.hist_base_time = hist_base_time
        b.hist_hours = hist_hours
        b.hist_device = hist_device
        b.tile_rules = int(tile_rules)
        b.flags = (_lib.OTR_BATCH_COPY_OUT if copy_out else 0) | (_lib.OTR_BATCH_TIMING if timing else 0) | \
            (_lib.OTR_BATCH_TILE_ROWS if tile_rows else 0) | (_lib.OTR_BATCH_COPY_REPORTS if copy_reports else 0) | \
            (_lib.OTR_BATCH_ROUTE_WORK if route_work else 0)
        r = _lib.BatchResult()
        rc = self._L.otr_match_batch(self._h, ctypes.byref(b), ctypes.byref(r))
        if rc != 0:
            raise RuntimeError('otr_match_batch failed (%d): %s' % (rc, _lib.last_error()))
        r._owner = self  # the host arrays belong to this matcher: keep it alive with the result
        return r

    def ingest(self, text, rules=0, separator='|', uuid_index=1, time_index=0, lat_index=9, lon_index=10,
               accuracy_index=5, time_format=None, inactivity=120, mode='auto', bbox=None, device_ptr=None,
               nbytes=None):
        """Probe text → windowed traces in HBM (include/otr.h otr_ingest).  text: bytes
        (host), or device_ptr + nbytes for text already in HBM.  Defaults: the raw-feed
        valuer and time pattern of simple_reporter.py:352-353.  Returns (IngestResult,
        batch) where batch is a device-array handle for match_batch(batch, device_arrays=
        batch.arrays).  Raises ValueError with the line number where the reference raises."""
        f = _lib.IngestFormat()
        f.rules = int(rules)
        f.separator = ord(separator) if isinstance(separator, str) else int(separator)
        f.uuid_index, f.time_index, f.lat_index, f.lon_index, f.accuracy_index = (
            uuid_index, time_index, lat_index, lon_index, accuracy_index)
        if time_format is None:
            time_format = _lib.OTR_TIME_EPOCH if rules == _lib.OTR_INGEST_SHARD else _lib.OTR_TIME_YMDHMS
        f.time_format = int(time_format)
        f.inactivity = int(inactivity)
        f.mode = {'auto': 0, 'bicycle': 1, 'pedestrian': 2}[mode] if isinstance(mode, str) else int(mode)
        if bbox is not None:
            f.use_bbox = 1
            for k in range(4):
                f.bbox[k] = float(bbox[k])
        r = _lib.IngestResult()
        if device_ptr is not None:
            rc = self._L.otr_ingest(self._h, ctypes.c_void_p(device_ptr), int(nbytes), _lib.OTR_MEM_DEVICE,
                                    ctypes.byref(f), ctypes.byref(r))
        else:
            self._keep = [text]
            rc = self._L.otr_ingest(self._h, ctypes.c_char_p(text), len(text), _lib.OTR_MEM_HOST, ctypes.byref(f),
                                    ctypes.byref(r))
        if rc != 0:
            if r.bad_line >= 0:
                raise ValueError('line %d: %s' % (r.bad_line, _lib.INGEST_REASONS.get(r.bad_reason, r.bad_reason)))
            raise RuntimeError('otr_ingest failed (%d): %s' % (rc, _lib.last_error()))
        return r, IngestedBatch(r)

    def match_batch_numpy(self, traces, **kw):
        r = self.match_batch(traces, copy_out=True, **kw)
        return _lib.result_to_numpy(r)
