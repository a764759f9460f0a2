"""One answer per trace (reporter_service.py:240): the same batch run again gives the
same output, field by field, through the shipped library — with the route kernels'
work counting on and off (the instrumented and the timed builds of every route kernel,
bench.py's two kinds of step), and whatever the run-to-run order of the work-queue
claims, the retry lists' task pairings and the dump-slot claims of the node and
edge-state retry tiers.  Workloads: C4's shape (60 s steps, 200 m radius: most searches
outgrow the first tables, dump and resume) and the deployed configuration (edge-state
searches with dumps).  tools/determinism.py is the full-size version."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GTT = {'turn_penalty_factor': 0, 'beta': 3, 'sigma_z': 4.07, 'breakage_distance': 2000}
CASES = {
    # traces, points, rate s, sigma m, seed, accuracy m, match options
    'c4': (2000, 60, 60, 50.0, 4, 50.0, dict(GTT, search_radius=200, max_search_radius=200, gps_accuracy=82.24)),
    'c2dep': (1000, 100, 15, 10.0, 2, None, {}),
}


@pytest.mark.parametrize('name', sorted(CASES))
def test_runs_identical(graph_dir, name):
    from reporter_amd import _lib
    from reporter_amd import matcher as M
    from reporter_amd.tools import gen
    nt, pts, rate, sig, seed, acc, opts = CASES[name]
    gp = gen.graph_path('metro', graph_dir)
    tr = gen.make_traces(gp, nt, pts, rate, sig, seed, 0.0, 0.0, acc)
    M.configure(M.default_config(gp, **opts))
    m = M.Matcher()
    from oracle.compare import compare
    outs, work = [], []
    for i in range(4):
        r = m.match_batch(tr, copy_out=True, tile_rows=True, route_work=bool(i & 1))
        assert r.status == 0, r.status
        o = _lib.result_to_numpy(r)
        outs.append({k: (np.array(v, copy=True) if isinstance(v, np.ndarray) else v) for k, v in o.items()})
        work.append([int(r.counters[k]) for k in (7, 11, 12, 22, 23)])
    # the instrumented runs did resume outgrown searches from their dumps
    assert work[1][1] + work[1][3] > 0, work
    for i in range(1, len(outs)):
        errors, stats = compare(outs[i], outs[0])  # (candidate arrays compared up to each count)
        assert not errors and all(stats.values()), (name, i, errors, stats)
        assert work[i][0] == work[0][0], work  # output segments
