// The reference's MapReduce triangle finder (oink/tri_find.cpp:43-82, the
// callbacks :104-325) as a reusable pipeline: 4 collates over the engine's
// generic ops, each stage timed. Used by the OINK command tri_find_mr and by
// bench.py's trifind_mr extras (the generic engine at large KV counts).
#pragma once
#include <string>
#include <vector>

#include "engine/mapreduce.h"

namespace mrh {
namespace oink {

struct TriMRStage {
  std::string op;       // "map_edge_vert", "collate 1", ...
  double seconds = 0;   // device-synchronised wall time of the op
  int64_t pairs_in = 0, pairs_out = 0;  // global pair counts before / after
  int64_t h2d_bytes = 0, d2h_bytes = 0;  // this rank's host <-> device copies during the op (xfer.h)
  int64_t disk_bytes = 0;                 // bytes this process wrote to spool / result files during the op
};
struct TriMRRun {
  uint64_t triangles = 0;
  int compact_vb = 0;  // > 0: the last collate ran on the compact layout (12-byte wedges)
  std::vector<TriMRStage> stages;
};

// mre: KV of EDGE{u64,u64} keys (NULL values), any distribution, unique and
// vi < vj (the output of edge_upper); mrt (empty, settings as wanted:
// budgets, fpath) ends with the triangles (vi, vj, vk). upper: first run
// edge_upper on mre in place (map edge_upper -> collate -> reduce cull,
// oink/edge_upper.cpp:37-60), for raw generated edges
TriMRRun tri_find_mr(MapReduce& mre, MapReduce& mrt, bool upper = false);

}  // namespace oink
}  // namespace mrh
