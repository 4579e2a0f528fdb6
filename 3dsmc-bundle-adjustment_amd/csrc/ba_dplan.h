// ba_dplan.h — the window plan's observation passes on the device (libmiba, internal).
//
// ba_prepare's host plan (ba_plan.cpp) makes four passes over the observations and a per-point sort; at C4
// (1M observations) they cost 2.1 ms on 16 host threads, 75 % of a new window's prepare. The raw observations are
// in HBM anyway (the device gather reads them), so the same orderings are built there, as integer passes with
// no host round trip between them, and ONE read-back hands the host what its sequential steps need (the greedy
// Schur tiles, the back-substitution chunks, the camera segments, the envelope): per-camera counts, the first
// co-visible cameras and, per active point in the point order, its observation count and camera range.
//
// Every ordering is the host plan's, element for element (a total order: stable bucket scatters in index order,
// per-point sorts on the unique key (active camera + 1, observation index)), so the plan arrays — and every
// solve — are bitwise those of the host plan (tests/test_gpu_plan.py compares their digests).
#pragma once
#include <hip/hip_runtime.h>

#include "ba_plan.h"

namespace miba {

static constexpr int DP_LONG_MAX = 4096;  // per-point list sorted in LDS (keys 32 KB)
static constexpr int DP_R = 1024;         // observations / points per bucket-scatter workgroup

struct DPlanArgs {
    // inputs (device): the raw window's indices and admissibility bytes (depth > 1e-15; the depths and pixels are
    // DMA'd on the copy stream while the passes run)
    const int* cam; const int* pt; const unsigned char* adm;
    int no, np, nc, fixed_cam, tile_win, chunk_obs;
    // outputs (device)
    int* po_dest;   // [no] original index -> point-major slot (-1: not admissible)
    int* co_dest;   // [no] original index -> camera-major slot (-1)
    int* cam_ac;    // [nc]
    int* pt_idx;    // [np] active point order (first n_ap)
    int* ovf_obs;   // [no] (first n_ovf)
    int* sum;       // read-back summary (ba_plan.h): [DP_HDR] | cam_cnt | fc | pt_ptr | first << 16 | last camera
    int* sum_host;  // device address of mapped host memory: the summary's live ranges are copied there last
    // scratch (device), dplan_scratch_ints() ints
    int* scratch;
};
size_t dplan_scratch_ints(int no, int np, int nc);
// the window fits the device plan (bucket histograms in LDS, the packed camera range of the summary)
bool dplan_fits(int no, int np, int nc);
// enqueue the passes on s; the summary is complete when s reaches the end of the enqueued work
hipError_t dplan_enqueue(const DPlanArgs& a, hipStream_t s);

}  // namespace miba
