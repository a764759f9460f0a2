"""Field-by-field parity check of a HIP batch result against the oracle — TEST
INFRASTRUCTURE ONLY (used by tests/ and __graft_entry__.smoke()).

Contract (BASELINE.json north_star): matched edge and OSMLR segment-id sequences
bit-exact; lengths, times and speeds within 1e-6 relative.  The implementation is
designed to be bit-exact everywhere, so floats are also compared exactly first and
only the tolerance is enforced.
"""
import numpy as np

REL_TOL = 1e-6


def _eq(name, a, b, errors):
    a = np.asarray(a)
    b = np.asarray(b)
    if a.shape != b.shape:
        errors.append('%s: shape %s vs %s' % (name, a.shape, b.shape))
        return False
    if not np.array_equal(a, b):
        idx = np.flatnonzero(a.reshape(-1) != b.reshape(-1))[:5]
        errors.append('%s: %d mismatches, first at %s: %s vs %s' % (
            name, int((a != b).sum()), idx.tolist(), a.reshape(-1)[idx].tolist(), b.reshape(-1)[idx].tolist()))
        return False
    return True


def _close(name, a, b, errors, stats):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    if a.shape != b.shape:
        errors.append('%s: shape %s vs %s' % (name, a.shape, b.shape))
        return
    exact = np.array_equal(a, b)
    stats[name + '_bitexact'] = bool(exact)
    if exact:
        return
    den = np.maximum(np.abs(b), 1e-300)
    rel = np.abs(a - b) / den
    bad = rel > REL_TOL
    if bad.any():
        i = np.flatnonzero(bad)[:5]
        errors.append('%s: %d values beyond %g rel, e.g. %s vs %s' % (name, int(bad.sum()), REL_TOL,
                                                                      a[i].tolist(), b[i].tolist()))


def compare(gpu, orc):
    """Returns (errors, stats).  Empty errors == parity."""
    errors, stats = [], {}
    for k in ('trace_state_off', 'state_probe', 'cand_count'):
        _eq(k, gpu[k], orc[k], errors)
    if errors:
        return errors, stats
    cnt = orc['cand_count']
    mask = np.arange(gpu['cand_edge'].shape[1])[None, :] < cnt[:, None]
    _eq('cand_edge', gpu['cand_edge'][mask], orc['cand_edge'][mask], errors)
    _close('cand_p', gpu['cand_p'][mask], orc['cand_p'][mask], errors, stats)
    _close('cand_sqd', gpu['cand_sqd'][mask], orc['cand_sqd'][mask], errors, stats)
    for k in ('winner', 'subpath', 'trace_route_off', 'route_edge', 'trace_seg_off', 'seg_id', 'seg_length',
              'seg_queue', 'seg_internal', 'seg_begin_shape', 'seg_end_shape', 'seg_way_off', 'seg_way',
              'trace_rep_off', 'rep_id', 'rep_next', 'rep_length', 'rep_queue', 'shape_used', 'stats'):
        _eq(k, gpu[k], orc[k], errors)
    for k in ('seg_start', 'seg_end', 'rep_t0', 'rep_t1', 'stats_len'):
        _close(k, gpu[k], orc[k], errors, stats)
    stats['n_states'] = int(len(orc['state_probe']))
    stats['n_seg'] = int(len(orc['seg_id']))
    stats['n_rep'] = int(len(orc['rep_id']))
    return errors, stats


def subset(res, idx, probe_off):
    """The results of traces `idx` (ascending) out of a batch result dict (GPU or oracle
    layout), re-based as if those traces had been matched alone: per-trace offsets
    restart at 0 and state_probe indexes the subset's own probes (probe_off: the
    batch's trace probe offsets).  A trace's results do not depend on the other traces
    of its batch, so subset(full batch) == match(subset) field by field."""
    idx = np.asarray(idx, dtype=np.int64)
    out = {}

    def take(off_key, keys):
        off = np.asarray(res[off_key], np.int64)
        parts = [np.arange(off[t], off[t + 1]) for t in idx]
        sel = np.concatenate(parts) if parts else np.zeros(0, np.int64)
        lens = np.array([off[t + 1] - off[t] for t in idx], np.int64)
        o = np.zeros(len(idx) + 1, np.int64)
        o[1:] = np.cumsum(lens)
        out[off_key] = o
        for k in keys:
            out[k] = np.asarray(res[k])[sel]
        return sel

    sel = take('trace_state_off', ('state_probe', 'cand_count', 'cand_edge', 'cand_p', 'cand_sqd', 'winner',
                                   'subpath'))
    # probe indices: global in the batch -> global in the subset
    po_ = np.asarray(probe_off, np.int64)
    lens = po_[idx + 1] - po_[idx]
    sub_off = np.zeros(len(idx) + 1, np.int64)
    sub_off[1:] = np.cumsum(lens)
    st_trace = np.repeat(np.arange(len(idx)), np.diff(out['trace_state_off']))
    out['state_probe'] = out['state_probe'] - po_[idx][st_trace] + sub_off[st_trace]
    take('trace_route_off', ('route_edge',))
    seg_sel = take('trace_seg_off', ('seg_id', 'seg_start', 'seg_end', 'seg_length', 'seg_queue', 'seg_internal',
                                     'seg_begin_shape', 'seg_end_shape'))
    wo = np.asarray(res['seg_way_off'], np.int64)
    wparts = [np.arange(wo[q], wo[q + 1]) for q in seg_sel]
    wsel = np.concatenate(wparts) if wparts else np.zeros(0, np.int64)
    wl = np.array([wo[q + 1] - wo[q] for q in seg_sel], np.int64)
    out['seg_way_off'] = np.concatenate([[0], np.cumsum(wl)]).astype(np.int64)
    out['seg_way'] = np.asarray(res['seg_way'])[wsel]
    take('trace_rep_off', ('rep_id', 'rep_next', 'rep_t0', 'rep_t1', 'rep_length', 'rep_queue'))
    out['shape_used'] = np.asarray(res['shape_used'])[idx]
    out['stats'] = np.asarray(res['stats'])[idx]
    out['stats_len'] = np.asarray(res['stats_len'])[idx]
    return out
