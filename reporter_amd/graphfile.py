"""Read-only numpy view of a flattened graph file (layout: include/otr_graph_format.h)."""
import struct

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
