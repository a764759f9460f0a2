"""Drop-in for the `valhalla` Python binding as the reference uses it.

    import reporter_amd.valhalla as valhalla
    valhalla.Configure(conf_path)                 # reporter_service.py:284, simple_reporter.py:132
    m = valhalla.SegmentMatcher()                 # reporter_service.py:52,  simple_reporter.py:133
    out = m.Match(json.dumps(trace))              # reporter_service.py:240, simple_reporter.py:166

Backed by libotr.so (HIP kernels on the MI355X); failures raise RuntimeError like the
boost.python binding's exceptions, which the callers catch (reporter_service.py:244,
simple_reporter.py:171).
"""
from . import matcher as _m


def Configure(conf_path):
    _m.configure(conf_path)


class SegmentMatcher(object):
    def __init__(self):
        self._m = _m.Matcher()

    def Match(self, trace_json):
        return self._m.match_json(trace_json)
