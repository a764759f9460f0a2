"""ctypes binding of libotr.so (include/otr.h).  No fallback: if the HIP library is
missing or cannot load, every entry point raises — the product never silently runs
anything else."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('OTR_LIB') or os.path.join(_HERE, 'libotr.so')
P = ctypes.POINTER

OTR_OK = 0
OTR_MEM_HOST = 0
OTR_MEM_DEVICE = 1
OTR_BATCH_COPY_OUT = 1
OTR_BATCH_TIMING = 2
OTR_BATCH_COPY_REPORTS = 4
OTR_BATCH_TILE_ROWS = 8
OTR_BATCH_ROUTE_WORK = 16
OTR_TILE_RULES_SIMPLE = 0
OTR_TILE_RULES_STREAM = 1
OTR_INGEST_SHARD = 0
OTR_INGEST_RAW = 1
OTR_INGEST_JAVA_SV = 2
OTR_TIME_EPOCH = 0
OTR_TIME_YMDHMS = 1
INGEST_REASONS = {1: 'fields', 2: 'float', 3: 'int', 4: 'time', 5: 'uuid', 6: 'precision', 7: 'collision',
                  8: 'accuracy'}
OTR_NO_ID = 0xFFFFFFFFFFFFFFFF
HIST_BINS = 8
KMAX = 64
STAGES = ['states', 'candidates', 'link', 'route', 'route_big', 'viterbi', 'paths', 'paths_big', 'segments',
          'histogram']

# every symbol include/otr.h declares
EXPORTS = ['otr_configure', 'otr_configure_json', 'otr_matcher_new', 'otr_matcher_free', 'otr_match',
           'otr_report', 'otr_report_segments', 'otr_free', 'otr_last_error', 'otr_match_batch',
           'otr_graph_info', 'otr_matcher_stream', 'otr_device', 'otr_report_batch', 'otr_coalesce',
           'otr_tiles_cull', 'otr_tiles_format', 'otr_ingest', 'otr_report_lists_device', 'otr_hist_reduce',
           'otr_tilehier_row', 'otr_tilehier_col', 'otr_tilehier_file', 'otr_tilehier_files', 'otr_flatten',
           'otr_max_batch_probes', 'otr_launch_max_items', 'otr_service_stats']


class ServiceSplit(ctypes.Structure):
    """otr_service_split (include/otr.h): the JSON request path's host split."""
    _fields_ = [('calls', ctypes.c_int64), ('items', ctypes.c_int64), ('device_batches', ctypes.c_int64),
                ('scan_s', ctypes.c_double), ('soa_s', ctypes.c_double), ('device_s', ctypes.c_double),
                ('format_s', ctypes.c_double), ('total_s', ctypes.c_double)]


class FlatGraph(ctypes.Structure):
    """otr_flat_graph (include/otr.h): decoded road-graph arrays for otr_flatten."""
    _fields_ = [('n_nodes', ctypes.c_uint32), ('node_ll', ctypes.c_void_p), ('n_edges', ctypes.c_uint32),
                ('edge_src', ctypes.c_void_p), ('edge_dst', ctypes.c_void_p), ('edge_attr', ctypes.c_void_p),
                ('edge_seg', ctypes.c_void_p), ('edge_way', ctypes.c_void_p), ('shape_off', ctypes.c_void_p),
                ('shape_ll', ctypes.c_void_p), ('n_segments', ctypes.c_uint32), ('seg_id', ctypes.c_void_p),
                ('seg_len', ctypes.c_void_p), ('cell_deg', ctypes.c_double)]


class FlatStats(ctypes.Structure):
    _fields_ = [('n_nodes', ctypes.c_uint32), ('n_edges', ctypes.c_uint32), ('n_contracted_edges', ctypes.c_uint32),
                ('n_merged_nodes', ctypes.c_uint32)]


class TraceBatch(ctypes.Structure):
    _fields_ = [('n_traces', ctypes.c_int32), ('memory', ctypes.c_int32),
                ('trace_offsets', ctypes.c_void_p), ('lat', ctypes.c_void_p), ('lon', ctypes.c_void_p),
                ('time', ctypes.c_void_p), ('accuracy', ctypes.c_void_p), ('mode', ctypes.c_void_p),
                ('report_levels', ctypes.c_uint32), ('transition_levels', ctypes.c_uint32),
                ('threshold_sec', ctypes.c_int32), ('quantisation', ctypes.c_int32),
                ('hist_base_time', ctypes.c_int64), ('hist_hours', ctypes.c_int32), ('flags', ctypes.c_int32),
                ('hist_device', ctypes.c_void_p), ('tile_rules', ctypes.c_int32), ('reserved', ctypes.c_int32)]


class IngestFormat(ctypes.Structure):
    _fields_ = [('rules', ctypes.c_int32), ('separator', ctypes.c_int32), ('uuid_index', ctypes.c_int32),
                ('time_index', ctypes.c_int32), ('lat_index', ctypes.c_int32), ('lon_index', ctypes.c_int32),
                ('accuracy_index', ctypes.c_int32), ('time_format', ctypes.c_int32), ('inactivity', ctypes.c_int32),
                ('mode', ctypes.c_int32), ('use_bbox', ctypes.c_int32), ('reserved', ctypes.c_int32),
                ('bbox', ctypes.c_double * 4)]


class IngestResult(ctypes.Structure):
    _fields_ = [('n_lines', ctypes.c_int64), ('n_kept', ctypes.c_int64), ('n_probes', ctypes.c_int64),
                ('n_traces', ctypes.c_int32), ('n_uuids', ctypes.c_int32), ('bad_line', ctypes.c_int64),
                ('bad_reason', ctypes.c_int32), ('parse_ms', ctypes.c_float), ('total_ms', ctypes.c_float),
                ('reserved', ctypes.c_int32), ('batch', TraceBatch),
                ('d_trace_uuid_off', ctypes.c_void_p), ('d_trace_uuid_len', ctypes.c_void_p)]


class BatchResult(ctypes.Structure):
    _fields_ = [('n_traces', ctypes.c_int32), ('n_probes', ctypes.c_int64), ('n_states', ctypes.c_int64),
                ('n_route', ctypes.c_int64), ('n_seg', ctypes.c_int64), ('n_rep', ctypes.c_int64),
                ('n_rows', ctypes.c_int64), ('status', ctypes.c_int32), ('n_overflow_traces', ctypes.c_int32),
                ('trace_state_off', P(ctypes.c_int64)), ('state_probe', P(ctypes.c_int64)),
                ('cand_count', P(ctypes.c_int32)), ('cand_edge', P(ctypes.c_uint32)),
                ('cand_p', P(ctypes.c_double)), ('cand_sqd', P(ctypes.c_double)),
                ('winner', P(ctypes.c_int32)), ('subpath', P(ctypes.c_int32)),
                ('trace_route_off', P(ctypes.c_int64)), ('route_edge', P(ctypes.c_uint32)),
                ('trace_seg_off', P(ctypes.c_int64)), ('seg_id', P(ctypes.c_uint64)),
                ('seg_start', P(ctypes.c_double)), ('seg_end', P(ctypes.c_double)),
                ('seg_length', P(ctypes.c_int32)), ('seg_queue', P(ctypes.c_int32)),
                ('seg_internal', P(ctypes.c_uint8)), ('seg_begin_shape', P(ctypes.c_int32)),
                ('seg_end_shape', P(ctypes.c_int32)), ('seg_way_off', P(ctypes.c_int64)),
                ('seg_way', P(ctypes.c_uint32)), ('trace_rep_off', P(ctypes.c_int64)),
                ('rep_id', P(ctypes.c_uint64)), ('rep_next', P(ctypes.c_uint64)),
                ('rep_t0', P(ctypes.c_double)), ('rep_t1', P(ctypes.c_double)),
                ('rep_length', P(ctypes.c_int32)), ('rep_queue', P(ctypes.c_int32)),
                ('shape_used', P(ctypes.c_int32)), ('stats', P(ctypes.c_int32)),
                ('stats_len', P(ctypes.c_double)), ('d_hist', ctypes.c_void_p), ('hist_len', ctypes.c_int64),
                ('counters', ctypes.c_uint64 * 24), ('kernel_ms', ctypes.c_float * 16),
                ('trace_status', P(ctypes.c_int32)), ('d_rows', ctypes.c_void_p),
                ('route_tier_code', ctypes.c_int32 * 16), ('route_tier_ms', ctypes.c_float * 16),
                ('route_tier_work', (ctypes.c_uint64 * 4) * 16)]


# otr_hist_entry (include/otr.h), 32 bytes
HIST_ENTRY = np.dtype([('file', '<u8'), ('id', '<u8'), ('next_id', '<u8'), ('speed_bin', '<u4'), ('count', '<u4')])

# otr_tile_row (include/otr.h), 56 bytes
TILE_ROW = np.dtype([('file', '<u8'), ('id', '<u8'), ('next_id', '<u8'), ('start', '<i8'), ('end', '<i8'),
                     ('duration', '<i4'), ('length', '<i4'), ('queue_length', '<i4'), ('speed_bin', '<i4')])


_L = None


def lib():
    """Load libotr.so once.  torch (if installed) is imported first so that the
    process holds a single HIP runtime (libotr links the one torch ships)."""
    global _L
    if _L is not None:
        return _L
    if not os.path.exists(LIB_PATH):
        raise RuntimeError('reporter_amd/libotr.so is not built: run `python __graft_entry__.py build` '
                           '(the HIP path has no fallback)')
    try:
        import torch  # noqa: F401  (shares its libamdhip64 with libotr)
    except Exception:
        pass
    L = ctypes.CDLL(LIB_PATH)
    L.otr_configure.argtypes = [ctypes.c_char_p]
    L.otr_configure_json.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
    L.otr_matcher_new.restype = ctypes.c_void_p
    L.otr_matcher_free.argtypes = [ctypes.c_void_p]
    L.otr_match.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, P(ctypes.c_void_p),
                            P(ctypes.c_size_t)]
    L.otr_report.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, P(ctypes.c_void_p),
                             P(ctypes.c_size_t)]
    L.otr_report_segments.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                      ctypes.c_int, P(ctypes.c_int32), ctypes.c_int, P(ctypes.c_int32),
                                      ctypes.c_int, P(ctypes.c_void_p), P(ctypes.c_size_t)]
    L.otr_free.argtypes = [ctypes.c_void_p]
    L.otr_last_error.restype = ctypes.c_char_p
    L.otr_match_batch.argtypes = [ctypes.c_void_p, P(TraceBatch), P(BatchResult)]
    L.otr_graph_info.argtypes = [P(ctypes.c_int64), P(ctypes.c_int64), P(ctypes.c_int64)]
    L.otr_matcher_stream.argtypes = [ctypes.c_void_p]
    L.otr_matcher_stream.restype = ctypes.c_void_p
    L.otr_report_batch.argtypes = [ctypes.c_void_p, ctypes.c_int32, P(ctypes.c_char_p), P(ctypes.c_size_t),
                                   ctypes.c_int, P(ctypes.c_int32), P(ctypes.c_void_p), P(ctypes.c_size_t)]
    L.otr_coalesce.argtypes = [ctypes.c_int32, ctypes.c_int32]
    if hasattr(L, 'otr_service_stats'):  # (an A/B build of an earlier round may lack it)
        L.otr_service_stats.argtypes = [P(ServiceSplit), ctypes.c_int]
    L.otr_tiles_cull.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                 ctypes.c_int32, P(ctypes.c_void_p), P(ctypes.c_int64)]
    L.otr_tiles_format.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_char_p, ctypes.c_char_p,
                                   ctypes.c_int32, P(ctypes.c_void_p), P(ctypes.c_size_t)]
    L.otr_ingest.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, P(IngestFormat),
                             P(IngestResult)]
    if hasattr(L, 'otr_max_batch_probes'):  # (an A/B build of an earlier round may lack them)
        L.otr_max_batch_probes.restype = ctypes.c_int64
        L.otr_launch_max_items.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int32]
        L.otr_launch_max_items.restype = ctypes.c_uint64
    L.otr_tilehier_row.argtypes = [ctypes.c_int32, ctypes.c_double]
    L.otr_tilehier_row.restype = ctypes.c_int32
    L.otr_tilehier_col.argtypes = [ctypes.c_int32, ctypes.c_double]
    L.otr_tilehier_col.restype = ctypes.c_int32
    L.otr_tilehier_file.argtypes = [ctypes.c_int32, ctypes.c_int64, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]
    L.otr_tilehier_files.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_char_p,
                                 P(ctypes.c_void_p), P(ctypes.c_size_t)]
    L.otr_flatten.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]
    L.otr_hist_reduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                  ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, P(ctypes.c_int64)]
    _L = L
    return L


def last_error():
    return lib().otr_last_error().decode('utf-8', 'replace')


def take_string(ptr, n):
    """Copy a library-owned output string and release it with otr_free."""
    if not ptr.value:
        return ''
    s = ctypes.string_at(ptr.value, n.value).decode('utf-8')
    lib().otr_free(ptr.value)
    return s


def levels_mask(levels):
    m = 0
    for l in levels:
        l = int(l)
        if 0 <= l < 32:
            m |= 1 << l
    return m


def _arr(p, n, dt):
    if n <= 0 or not p:
        return np.zeros(max(n, 0), dt)
    return np.ctypeslib.as_array(p, shape=(n,)).astype(dt, copy=True)


def result_to_numpy(r):
    """Host arrays of an OTR_BATCH_COPY_OUT result (same keys as oracle.pyoracle.match_batch)."""
    nt, ns, nseg, nrep = r.n_traces, r.n_states, r.n_seg, r.n_rep
    out = dict(
        trace_state_off=_arr(r.trace_state_off, nt + 1, np.int64),
        state_probe=_arr(r.state_probe, ns, np.int64),
        cand_count=_arr(r.cand_count, ns, np.int32),
        cand_edge=_arr(r.cand_edge, ns * KMAX, np.uint32).reshape(ns, KMAX),
        cand_p=_arr(r.cand_p, ns * KMAX, np.float64).reshape(ns, KMAX),
        cand_sqd=_arr(r.cand_sqd, ns * KMAX, np.float64).reshape(ns, KMAX),
        winner=_arr(r.winner, ns, np.int32), subpath=_arr(r.subpath, ns, np.int32),
        trace_route_off=_arr(r.trace_route_off, nt + 1, np.int64),
        route_edge=_arr(r.route_edge, r.n_route, np.uint32),
        trace_seg_off=_arr(r.trace_seg_off, nt + 1, np.int64),
        seg_id=_arr(r.seg_id, nseg, np.uint64), seg_start=_arr(r.seg_start, nseg, np.float64),
        seg_end=_arr(r.seg_end, nseg, np.float64), seg_length=_arr(r.seg_length, nseg, np.int32),
        seg_queue=_arr(r.seg_queue, nseg, np.int32), seg_internal=_arr(r.seg_internal, nseg, np.uint8),
        seg_begin_shape=_arr(r.seg_begin_shape, nseg, np.int32),
        seg_end_shape=_arr(r.seg_end_shape, nseg, np.int32),
        seg_way_off=_arr(r.seg_way_off, nseg + 1, np.int64),
        trace_rep_off=_arr(r.trace_rep_off, nt + 1, np.int64),
        rep_id=_arr(r.rep_id, nrep, np.uint64), rep_next=_arr(r.rep_next, nrep, np.uint64),
        rep_t0=_arr(r.rep_t0, nrep, np.float64), rep_t1=_arr(r.rep_t1, nrep, np.float64),
        rep_length=_arr(r.rep_length, nrep, np.int32), rep_queue=_arr(r.rep_queue, nrep, np.int32),
        shape_used=_arr(r.shape_used, nt, np.int32),
        stats=_arr(r.stats, nt * 7, np.int32).reshape(nt, 7),
        stats_len=_arr(r.stats_len, nt * 2, np.float64).reshape(nt, 2),
    )
    out['seg_way'] = _arr(r.seg_way, int(out['seg_way_off'][-1]) if nseg else 0, np.uint32)
    out['counters'] = list(r.counters)
    out['n_rows'] = r.n_rows
    out['status'] = r.status
    out['n_overflow'] = r.n_overflow_traces
    return out


def service_stats(reset=False):
    """otr_service_stats: the JSON path's host split since the last reset (dict)."""
    st = ServiceSplit()
    lib().otr_service_stats(ctypes.byref(st), 1 if reset else 0)
    return {k: getattr(st, k) for k, _ in ServiceSplit._fields_}
