// kernels.h — gfx950 (CDNA4, wave64) device code of libmaxcover.
//
// Hot path: one MADS poll = K candidates x full coverage of the fire-point list
// (src/TDM_STATIC_opt.jl:82-100 via src/AreaCoverageCalculation.jl:63-78), as a short chain:
//   disk_prep_kernel      (streaming scan) per (candidate, disk): {cx, cy, T(r), r}, T the exact
//                         threshold
//   prep_kernel           one pass over the 3N x K candidate matrix (or the LTMADS generator):
//                         the penalty chains + cons3 (vp per candidate), the packed integer
//                         keys (one row per disk), and a packed tile-range record per
//                         (workgroup, disk)
//   disk_index_kernel     (tiled / poll walks) per disk over all K candidates: the distinct disks
//                         (records), the candidate -> distinct map, the region and the two walk
//                         costs reduced from the prep's records, row descriptors, lane constants
//   walk_setup_kernel     per disk i the lower-index disks whose regions overlap region i (the
//                         poll-level neighbour lists every walk uses)
//   coverage_tiled_poll_kernel  (when forced, or AUTO chose it on the lane's recent polls) the
//                         walk choice with the lists known, then the per-candidate walk over
//                         (candidate x slice) units, pairs from the poll-level lists
//   coverage_poll_kernel  workgroup = disk i: the entries of disk i's region staged in LDS once,
//                         every wave holding all of the disk's distinct disks (8 per lane) over a
//                         quarter of the entries, exact fp32 filter; further workgroups run the
//                         shared-entry pass (fp64 jobs); shared_bits_kernel on crowded polls
//   coverage_tiled_kernel workgroup = candidate: each wave walks whole disks over the CSR rows
//                         (batches too small for the poll walk)
//   coverage_scan_kernel  streaming brute force (every entry x every disk), the fallback
//   finalize_kernel       fixed-order sum of per-disk credits (per position, gathered through the
//                         map) -> area, objective, and the argmin by the last-arriving block
//   closure_kernel        one candidate in one launch (the per-trial-point objective callback)
// (Cross-workgroup hand-offs use agent-scope stores drained before one counter add, never a
// device-scope fence: that fence writes back the XCD's L2 on gfx950.)
// An entry is credited to the LOWEST-index disk covering it (exactly-once union count), so the
// area is the reference's first-hit-break sum (:67-78) over the same multiset of entries.
// Partials are summed in disk (slice) order per candidate: bit-reproducible.
#pragma once

#include "k_common.h"
#include "k_prep.h"
#include "k_index.h"
#include "k_walk.h"
#include "k_poll.h"
#include "k_final.h"
#include "k_setup.h"
#include "k_closure.h"
#include "k_fiw.h"
