/*
 * otr_graph_format.h — on-disk / in-HBM layout of the flattened road graph.
 *
 * Valhalla/OSMLR routing tiles (UPSTREAM baldr GraphTile: nodes, directed edges,
 * edge shapes, way ids, traffic/OSMLR associations; tile hierarchy
 * /root/reference/py/get_tiles.py:30-102) are flattened ONCE into this single
 * binary file: a CSR road graph plus a uniform lat/lon grid edge index.  The
 * same arrays are uploaded verbatim to HBM by otr_configure() (include/otr.h),
 * one replica per GPU.  Plain C, little-endian, every array 64-byte aligned.
 *
 *   header (struct otr_graph_header, 256 bytes)
 *   node_row   u32[n_nodes+1]       CSR offsets of out-edges (edges sorted by src)
 *   node_ll    i32[2*n_nodes]       (lat_e6, lon_e6) micro-degrees
 *   rev_row    u32[n_nodes+1]       CSR offsets of in-edges
 *   rev_edge   u32[n_edges]         in-edge ids grouped by dst
 *   edge_src   u32[n_edges]
 *   edge_dst   u32[n_edges]
 *   edge_len   f32[n_edges]         metres (authoritative routing length)
 *   edge_attr  u32[n_edges]         OTR_ATTR_* bit fields below
 *   edge_shape u32[n_edges+1]       offsets into shape_ll (shape includes both end nodes)
 *   edge_seg   u32[n_edges]         OSMLR segment index, OTR_NO_SEGMENT if unassociated
 *   edge_way   u32[n_edges]         OSM way id (low 32 bits)
 *   shape_ll   i32[2*n_shape]       (lat_e6, lon_e6)
 *   seg_id     u64[n_segments]      OSMLR 64-bit id: level(3) | tile(22) | index(21)
 *                                   (simple_reporter.py:36-49)
 *   seg_len    u32[n_segments]      OSMLR segment length, whole metres
 *   cell_row   u32[n_cells+1]       grid CSR: cell = row*grid_cols + col
 *   cell_edge  u32[n_cell_entries]  edge ids whose shape touches the cell
 *
 * Grid cell of (lat, lon):  row = floor((lat - grid_min_lat) / grid_cell_deg),
 *                           col = floor((lon - grid_min_lon) / grid_cell_deg).
 * An edge is listed in every cell its shape's segment bounding boxes, padded by
 * OTR_GRID_PAD_DEG, overlap.  (Valhalla's meili grid: 500 cells per 0.25° tile
 * side => 0.0005°, the default cell size here.)
 */
#ifndef OTR_GRAPH_FORMAT_H
#define OTR_GRAPH_FORMAT_H

#include <stdint.h>

#define OTR_GRAPH_MAGIC   "OTRGRPH1"
#define OTR_GRAPH_VERSION 1u
#define OTR_NO_SEGMENT    0xFFFFFFFFu
#define OTR_GRID_PAD_DEG  1e-7

/* edge_attr bit fields */
#define OTR_ACCESS_AUTO        1u
#define OTR_ACCESS_BICYCLE     2u
#define OTR_ACCESS_PEDESTRIAN  4u
#define OTR_ATTR_ACCESS_MASK   0x7u
#define OTR_ATTR_SPEED_SHIFT   3          /* 8 bits, km/h */
#define OTR_ATTR_LEVEL_SHIFT   11         /* 3 bits, road hierarchy level 0..2 */
#define OTR_ATTR_INTERNAL      (1u << 14) /* intersection-internal / turn channel / roundabout */
#define OTR_ATTR_SEG_BEGIN     (1u << 15) /* edge starts its OSMLR segment */
#define OTR_ATTR_SEG_END       (1u << 16) /* edge ends its OSMLR segment */

#define OTR_ATTR_SPEED(a) (((a) >> OTR_ATTR_SPEED_SHIFT) & 0xFFu)
#define OTR_ATTR_LEVEL(a) (((a) >> OTR_ATTR_LEVEL_SHIFT) & 0x7u)

typedef struct otr_graph_header {
  char     magic[8];
  uint32_t version;
  uint32_t flags;
  uint32_t n_nodes;
  uint32_t n_edges;
  uint32_t n_shape;
  uint32_t n_segments;
  uint32_t n_cells;
  uint32_t n_cell_entries;
  uint32_t grid_rows;
  uint32_t grid_cols;
  double   grid_min_lat;
  double   grid_min_lon;
  double   grid_cell_deg;
  uint64_t array_offset[17];   /* byte offset of each array, in the order listed above */
  uint8_t  reserved[256 - 72 - 17 * 8];
} otr_graph_header;

enum otr_graph_array {
  OTR_A_NODE_ROW = 0, OTR_A_NODE_LL, OTR_A_REV_ROW, OTR_A_REV_EDGE, OTR_A_EDGE_SRC,
  OTR_A_EDGE_DST, OTR_A_EDGE_LEN, OTR_A_EDGE_ATTR, OTR_A_EDGE_SHAPE, OTR_A_EDGE_SEG,
  OTR_A_EDGE_WAY, OTR_A_SHAPE_LL, OTR_A_SEG_ID, OTR_A_SEG_LEN, OTR_A_CELL_ROW,
  OTR_A_CELL_EDGE, OTR_A_END
};

#endif
