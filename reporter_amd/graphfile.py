"""Read-only numpy view of a flattened graph file (layout: include/otr_graph_format.h)."""
import struct

import os

import numpy as np

_HDR = struct.Struct('<8sII8I3d17Q')
ARRAYS = [
    ('node_row', np.uint32, lambda h: h['n_nodes'] + 1),
    ('node_ll', np.int32, lambda h: 2 * h['n_nodes']),
    ('rev_row', np.uint32, lambda h: h['n_nodes'] + 1),
    ('rev_edge', np.uint32, lambda h: h['n_edges']),
    ('edge_src', np.uint32, lambda h: h['n_edges']),
    ('edge_dst', np.uint32, lambda h: h['n_edges']),
    ('edge_len', np.float32, lambda h: h['n_edges']),
    ('edge_attr', np.uint32, lambda h: h['n_edges']),
    ('edge_shape', np.uint32, lambda h: h['n_edges'] + 1),
    ('edge_seg', np.uint32, lambda h: h['n_edges']),
    ('edge_way', np.uint32, lambda h: h['n_edges']),
    ('shape_ll', np.int32, lambda h: 2 * h['n_shape']),
    ('seg_id', np.uint64, lambda h: h['n_segments']),
    ('seg_len', np.uint32, lambda h: h['n_segments']),
    ('cell_row', np.uint32, lambda h: h['n_cells'] + 1),
    ('cell_edge', np.uint32, lambda h: h['n_cell_entries']),
]
NO_SEGMENT = 0xFFFFFFFF
ATTR_INTERNAL = 1 << 14
ATTR_SEG_BEGIN = 1 << 15
ATTR_SEG_END = 1 << 16


class GraphFile:
    def __init__(self, path):
        self.path = path
        mm = np.memmap(path, dtype=np.uint8, mode='r')
        v = _HDR.unpack_from(mm[:_HDR.size].tobytes(), 0)
        if v[0] != b'OTRGRPH1':
            raise ValueError('%s: not an OTR graph file' % path)
        names = ['n_nodes', 'n_edges', 'n_shape', 'n_segments', 'n_cells', 'n_cell_entries', 'grid_rows',
                 'grid_cols']
        self.h = dict(zip(names, v[3:11]))
        self.h.update(grid_min_lat=v[11], grid_min_lon=v[12], grid_cell_deg=v[13])
        self.offsets = v[14:31]
        for i, (name, dt, cnt) in enumerate(ARRAYS):
            n = cnt(self.h)
            setattr(self, name, np.frombuffer(mm, dtype=dt, count=n, offset=self.offsets[i]))
        self.n_nodes = self.h['n_nodes']
        self.n_edges = self.h['n_edges']


def _cos_deg(deg):
    import math
    return math.cos(math.radians(deg))


def write_graph(path, node_ll, edges, segments=(), cell_deg=0.0005):
    """Flatten an explicit road graph into the OTR graph file.

    node_ll:  [(lat, lon)] in degrees (stored as micro-degrees)
    edges:    [dict(src, dst, shape=[(lat,lon),...] (interior points, optional),
                    speed=50, access=7, level=2, internal=False, way=1,
                    length=metres (optional; default: the polyline's length, at least 0.5 m))]
    segments: [dict(id=osmlr_id, edges=[edge indices in order])]  (length = sum of edge lengths)
    Edge ids in the file follow the CSR order (sorted by src, dst, input order);
    returns the permutation new_id_of[input_index].
    """
    import math
    M = 20037581.187 / 180.0
    node_ll = np.asarray(node_ll, dtype=np.float64)
    n_nodes = len(node_ll)
    nll = np.round(node_ll * 1e6).astype(np.int32)
    order = sorted(range(len(edges)), key=lambda i: (edges[i]['src'], edges[i]['dst'], i))
    new_id = np.empty(len(edges), np.int64)
    for nid, i in enumerate(order):
        new_id[i] = nid
    E = len(edges)
    node_row = np.zeros(n_nodes + 1, np.uint32)
    src = np.zeros(E, np.uint32)
    dst = np.zeros(E, np.uint32)
    elen = np.zeros(E, np.float32)
    attr = np.zeros(E, np.uint32)
    eshape = np.zeros(E + 1, np.uint32)
    eseg = np.full(E, NO_SEGMENT, np.uint32)
    eway = np.zeros(E, np.uint32)
    shape = []
    for nid, i in enumerate(order):
        e = edges[i]
        src[nid], dst[nid] = e['src'], e['dst']
        node_row[e['src'] + 1] += 1
        pts = [tuple(nll[e['src']])] + [tuple(np.round(np.asarray(p) * 1e6).astype(np.int32))
                                        for p in e.get('shape', [])] + [tuple(nll[e['dst']])]
        eshape[nid] = len(shape)
        L = 0.0
        for k, p in enumerate(pts):
            shape.append(p)
            if k:
                a, b = pts[k - 1], p
                la1, lo1, la2, lo2 = a[0] * 1e-6, a[1] * 1e-6, b[0] * 1e-6, b[1] * 1e-6
                x = (lo1 - lo2) * M * _cos_deg(0.5 * (la1 + la2))
                y = (la1 - la2) * M
                L += math.sqrt(x * x + y * y)
        elen[nid] = e['length'] if 'length' in e else max(L, 0.5)
        a = (e.get('access', 7) & 7) | (int(e.get('speed', 50)) << 3) | (int(e.get('level', 2)) << 11)
        if e.get('internal'):
            a |= ATTR_INTERNAL
        attr[nid] = a
        eway[nid] = e.get('way', 1)
    eshape[E] = len(shape)
    node_row = np.cumsum(node_row).astype(np.uint32)
    seg_id = np.zeros(len(segments), np.uint64)
    seg_len = np.zeros(len(segments), np.uint32)
    for si, s in enumerate(segments):
        ids = [int(new_id[i]) for i in s['edges']]
        seg_id[si] = s['id']
        seg_len[si] = int(round(sum(float(elen[x]) for x in ids)))
        for k, x in enumerate(ids):
            eseg[x] = si
            if k == 0:
                attr[x] |= ATTR_SEG_BEGIN
            if k == len(ids) - 1:
                attr[x] |= ATTR_SEG_END
    rev_row = np.zeros(n_nodes + 1, np.uint32)
    for x in dst:
        rev_row[x + 1] += 1
    rev_row = np.cumsum(rev_row).astype(np.uint32)
    rev_edge = np.zeros(E, np.uint32)
    fill = rev_row[:-1].astype(np.int64).copy()
    for x in range(E):
        rev_edge[fill[dst[x]]] = x
        fill[dst[x]] += 1
    shape_ll = np.asarray(shape, np.int32).reshape(-1)
    lat = shape_ll[0::2] * 1e-6
    lon = shape_ll[1::2] * 1e-6
    gmin_lat = math.floor(lat.min() / cell_deg) * cell_deg - cell_deg
    gmin_lon = math.floor(lon.min() / cell_deg) * cell_deg - cell_deg
    rows = int(math.ceil((lat.max() - gmin_lat) / cell_deg)) + 2
    cols = int(math.ceil((lon.max() - gmin_lon) / cell_deg)) + 2
    pad = 1e-7
    cells = [[] for _ in range(rows * cols)]
    for x in range(E):
        seen = set()
        for k in range(int(eshape[x]), int(eshape[x + 1]) - 1):
            la0, lo0 = shape_ll[2 * k] * 1e-6, shape_ll[2 * k + 1] * 1e-6
            la1, lo1 = shape_ll[2 * k + 2] * 1e-6, shape_ll[2 * k + 3] * 1e-6
            r0 = int(math.floor((min(la0, la1) - pad - gmin_lat) / cell_deg))
            r1 = int(math.floor((max(la0, la1) + pad - gmin_lat) / cell_deg))
            c0 = int(math.floor((min(lo0, lo1) - pad - gmin_lon) / cell_deg))
            c1 = int(math.floor((max(lo0, lo1) + pad - gmin_lon) / cell_deg))
            for r in range(max(r0, 0), min(r1, rows - 1) + 1):
                for c in range(max(c0, 0), min(c1, cols - 1) + 1):
                    seen.add(r * cols + c)
        for c in seen:
            cells[c].append(x)
    cell_row = np.zeros(rows * cols + 1, np.uint32)
    cell_edge = []
    for c in range(rows * cols):
        lst = sorted(cells[c])
        cell_edge.extend(lst)
        cell_row[c + 1] = cell_row[c] + len(lst)
    cell_edge = np.asarray(cell_edge, np.uint32)
    arrays = [node_row, nll.reshape(-1), rev_row, rev_edge, src, dst, elen, attr, eshape, eseg, eway, shape_ll,
              seg_id, seg_len, cell_row, cell_edge]
    offs = []
    blob = bytearray(256)
    for a in arrays:
        blob += b'\0' * ((-len(blob)) % 64)
        offs.append(len(blob))
        blob += np.ascontiguousarray(a).tobytes()
    offs.append(len(blob))
    hdr = _HDR.pack(b'OTRGRPH1', 1, 0, n_nodes, E, len(shape), len(segments), rows * cols, len(cell_edge),
                    rows, cols, gmin_lat, gmin_lon, cell_deg, *offs)
    blob[:_HDR.size] = hdr
    # written beside the target and renamed over it: a reader (another test process
    # building the same graph) never sees a partial file
    tmp = '%s.%d.tmp' % (path, os.getpid())
    with open(tmp, 'wb') as f:
        f.write(bytes(blob))
    os.replace(tmp, path)
    return new_id
