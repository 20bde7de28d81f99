// kernels.h — gfx950 (CDNA4, wave64) device code of libmaxcover.
//
// Hot path: one MADS poll = K candidates x full coverage of the fire-point list
// (src/TDM_STATIC_opt.jl:82-100 via src/AreaCoverageCalculation.jl:63-78), as a short chain:
//   disk_prep_kernel      (streaming scan) per (candidate, disk): {cx, cy, T(r), r}, T the exact
//                         threshold, and the objective-penalty term / cons3 mark
//   cands_keys_kernel     (matrix source) fp32 keys of every candidate value, variable-major
//   disk_index_kernel     (tiled / poll walks) per disk over all K candidates: the distinct disks
//                         (records, penalty terms), the candidate -> distinct map, the region
//                         and the two walk costs
//   walk_setup_kernel     the walk choice (every block; block 0 stores it), then per disk i the
//                         lower-index disks whose regions overlap region i (poll walk), or the
//                         per-candidate walk itself (grid-stride over candidate x slice units)
//   coverage_poll_kernel  workgroup = disk i: the entries of disk i's region staged in LDS once,
//                         every wave holding all of the disk's distinct disks (8 per lane) over a
//                         quarter of the entries, exact fp32 filter; further workgroups run the
//                         shared-entry pass and the penalty chains
//   coverage_tiled_kernel workgroup = candidate: each wave walks whole disks over the CSR rows
//                         (batches too small for the poll walk)
//   coverage_scan_kernel  streaming brute force (every entry x every disk), the fallback
//   finalize_kernel       fixed-order sum of per-slice partials -> area, objective
//   closure_kernel        one candidate in one launch (the per-trial-point objective callback)
// (Completion-counter "last block" fusions of decide/argmin were measured slower: the
// device-scope fence each block needs writes back its XCD's L2 on gfx950.)
// An entry is credited to the LOWEST-index disk covering it (exactly-once union count), so the
// area is the reference's first-hit-break sum (:67-78) over the same multiset of entries.
// Partials are laid out [slice][candidate] and summed in slice order: bit-reproducible.
#pragma once

#include "k_common.h"
#include "k_prep.h"
#include "k_index.h"
#include "k_walk.h"
#include "k_poll.h"
#include "k_final.h"
#include "k_setup.h"
#include "k_closure.h"
