"""Mirror of py/reporter_service.py's programmatic surface over libotr.

  report(segments, trace, threshold_sec, report_levels, transition_levels)
        reporter_service.py:79-179 — computed by the C++ report() shared with the
        device segment scan (reporter_amd/csrc/otr_report.h).
  handle_request(body) -> (code, body)
        reporter_service.py:209-245 — validation + Match + report() in one C-ABI call
        (otr_report), the call that replaces Batch.java:68's HTTP POST.
  handle_requests(bodies) -> [(code, body)]
        many bodies in shared device batches (otr_report_batch).
  serve(address, config, coalesce_traces)
        optional HTTP front (POST/GET /report) for callers that still speak HTTP;
        concurrent requests coalesce into shared device batches (otr_coalesce).
"""
import ctypes
import json
import os
import threading

from . import _lib
from . import matcher as _m

_local = threading.local()


def _threshold():
    t = os.environ.get('THRESHOLD_SEC')  # reporter_service.py:55-58
    return int(t) if t else 15


def _matcher():
    m = getattr(_local, 'matcher', None)
    if m is None:
        m = _m.Matcher()
        _local.matcher = m
    return m


def report(segments, trace, threshold_sec, report_levels, transition_levels):
    """report() of reporter_service.py:79-179 over a Match() result dict."""
    L = _lib.lib()
    mj = json.dumps(segments, separators=(',', ':')).encode()
    tj = json.dumps({'trace': trace['trace']}, separators=(',', ':')).encode()
    rl = sorted(int(x) for x in report_levels)
    tl = sorted(int(x) for x in transition_levels)
    ra = (ctypes.c_int32 * max(len(rl), 1))(*rl)
    ta = (ctypes.c_int32 * max(len(tl), 1))(*tl)
    out, n = ctypes.c_void_p(), ctypes.c_size_t()
    rc = L.otr_report_segments(mj, len(mj), tj, len(tj), int(threshold_sec), ra, len(rl), ta, len(tl),
                               ctypes.byref(out), ctypes.byref(n))
    body = _lib.take_string(out, n)
    if rc != 0:
        raise RuntimeError(body)
    return json.loads(body)


def handle_request(body, threshold_sec=None):
    """(code, body) as SegmentMatcherHandler.handle_request returns them."""
    t = _threshold() if threshold_sec is None else threshold_sec
    return _matcher().report_json(body, t)


def handle_requests(bodies, threshold_sec=None):
    """[(code, body)] for many POST /report bodies, matched in shared device batches."""
    t = _threshold() if threshold_sec is None else threshold_sec
    return _matcher().report_json_batch(bodies, t)


def serve(address, config, coalesce_traces=0, coalesce_wait_us=2000):
    """coalesce_traces > 0: concurrent requests of the server threads share device
    batches (otr_coalesce) instead of one device batch per request."""
    from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
    from urllib.parse import parse_qs, urlsplit
    _m.configure(config)
    if coalesce_traces > 0:
        _m.coalesce(coalesce_traces, coalesce_wait_us)

    class H(BaseHTTPRequestHandler):
        def _do(self, post):
            split = urlsplit(self.path)
            if split.path.split('/')[-1] != 'report':
                code, body = 400, '{"error":"Try a valid action: [\'report\']"}'
            elif post:
                code, body = handle_request(self.rfile.read(int(self.headers['Content-Length'])))
            else:
                q = parse_qs(split.query)
                code, body = handle_request(q['json'][0]) if 'json' in q else (400, '{"error":"No json provided"}')
            b = body.encode()
            self.send_response(code)
            self.send_header('Access-Control-Allow-Origin', '*')
            self.send_header('Content-type', 'application/json;charset=utf-8')
            self.send_header('Content-length', str(len(b)))
            self.end_headers()
            self.wfile.write(b)

        def do_GET(self):
            self._do(False)

        def do_POST(self):
            self._do(True)

    host, port = address.split('/')[-1].split(':')
    ThreadingHTTPServer((host, int(port)), H).serve_forever()
