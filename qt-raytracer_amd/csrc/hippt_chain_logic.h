// hippt_chain_logic.h — the integer rules of chained batches (hippt_trace.h "chained batches",
// DESIGN.md §7) as pure functions: which batches a launch combines and traces, what its waves learn
// from the host mailbox, and the frame offset a wave traces a batch with.  The gfx950 kernels call
// them; tests/native/chain_model.cpp compiles this header with g++ and drives the protocol through
// adversarial host/device interleavings (tests/test_chain_protocol.py).
//
// The anchor is the reference's frame-ordered accumulation: one launch and one sync per frame,
// every frame's sample blended into the running average in frame order
// (CudaPathTracerKernel.cu:157-178, 246-265).  A chained batch must therefore be traced exactly
// once, with the frames the host gave it, and combined exactly once, after every earlier batch.
#pragma once

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define HIPPT_CL __host__ __device__ __forceinline__
#else
#define HIPPT_CL inline
#endif

namespace hippt {
namespace chain {

// ---- the host mailbox word (pinned, coherent; written by chain_batch when a batch is posted) ----
// run << 33 | consecutive frames << 32 | last posted batch
HIPPT_CL unsigned long long box_word(unsigned run, bool consecutive, unsigned last) {
    return ((unsigned long long)run << 33) | ((unsigned long long)(consecutive ? 1u : 0u) << 32) | last;
}

// ---- a block's view of the mailbox (LDS ChainView: last, flags) ---------------------------------
// kConsec: batch t + 1 renders the frames after batch t's (else the same frames again);
// kClosed: the host is on a later run (no batch after `last` will be posted);
// kStepKnown: kConsec is meaningful.  The host knows the run's frame pattern from its second batch
// on (chain_batch: seq 1 sets the step), so a view that knows any batch >= 1 is posted knows it.
constexpr unsigned kConsec = 1u, kClosed = 2u, kStepKnown = 4u;

// The view a launch starts with: batches up to `posted` (chainPosted) posted, its step chainStep
// (-1: not known when the launch was enqueued, which happens only for a run's batch 0).
HIPPT_CL unsigned view_flags_at_start(int step) {
    return step < 0 ? 0u : (kStepKnown | (step > 0 ? kConsec : 0u));
}

// The per-XCD device copy of the mailbox word: refresh stamp (16-tick units) << 40 | launch epoch
// mod 64 << 34 | closed << 33 | (an open run's) consecutive << 32 | last posted batch.  A host word
// of another run makes the copy "closed" and carries nothing else: the word's batch and frame
// pattern are the later run's.
HIPPT_CL unsigned long long copy_pack(unsigned long long now, unsigned long long h, unsigned run, unsigned ep) {
    const bool closed = unsigned(h >> 33) != run;
    return ((now >> 4) << 40) | ((unsigned long long)(ep & 63u) << 34) |
           (closed ? (1ull << 33) : (h & ((1ull << 33) - 1ull)));
}
HIPPT_CL bool copy_closed(unsigned long long c) { return ((c >> 33) & 1ull) != 0ull; }
HIPPT_CL unsigned copy_last(unsigned long long c) { return unsigned(c); }

// Merges a copy into a view.  Monotone: `last` never decreases and no flag is ever cleared, so a
// wave that reads the view's two words at any moment sees a pair some merge produced or a later
// `flags` beside an earlier `last`, and both say only true things.  A closed copy adds kClosed and
// nothing else; an open copy that knows a batch >= 1 is posted carries the run's frame pattern.
// (Round 5 replaced `flags` by the copy's: a closed copy then cleared kConsec while `last` kept a
// posted batch, and a wave that moved into that batch traced it with frame offset 0 — the
// GPUTEST_r05 failure, tests/native/chain_model.cpp legacy_view_merge.)
HIPPT_CL void view_merge(unsigned &last, unsigned &flags, unsigned long long c) {
    if (copy_closed(c)) {
        flags |= kClosed;
        return;
    }
    const unsigned cl = copy_last(c);
    if (cl > last) last = cl;
    if (cl >= 1u) flags |= kStepKnown | unsigned((c >> 32) & 1ull);
}

// chain_next's answer for batch nt from a view: posted (and the run's step known) or not.  A view
// that does not know the step never lets a wave take a batch: that batch's own launch traces it.
HIPPT_CL bool view_takes(unsigned nt, unsigned last, unsigned flags, int frames, int &step) {
    if (nt > last || !(flags & kStepKnown)) return false;
    step = (flags & kConsec) ? frames : 0;
    return true;
}

// ---- a launch's plan at its start (chain_begin) ------------------------------------------------
// Ring-slot marker of the last launch that moved into a slot's batch: batch << 32 | epoch + 1.
HIPPT_CL unsigned long long marker(unsigned t, unsigned epoch) { return ((unsigned long long)t << 32) | (epoch + 1u); }
// Batch t finished by a launch before this one (epoch e): an earlier launch took it, and every
// earlier launch has ended before this one started.
HIPPT_CL bool marker_finished(unsigned long long m, unsigned t, unsigned e) {
    const unsigned by = unsigned(m);
    return unsigned(m >> 32) == t && by != 0u && by <= e;
}
// Lane k of chain_begin's ballot looks at batch t0 + k when it is inside the ring's window.
HIPPT_CL bool begin_lane_in_window(unsigned k, unsigned t0, unsigned c0, unsigned slots) {
    return k < slots && t0 + k < c0 + slots;
}

struct BeginPlan {
    unsigned t0;    // the first batch whose marker the launch reads
    int c1;         // the launch combines [c0, c1] (none when c1 < c0)
    unsigned u;     // the first batch it traces
    unsigned tLim;  // the last batch it may trace
};
// c0: the first batch not combined by an earlier launch; own: chainSeq; nfin: the marked batches
// from t0 on (the run of finished batches the ballot found); slots: the ring; cap: chainCap.
HIPPT_CL unsigned begin_t0(unsigned c0, unsigned own) { return own > c0 ? own : c0; }
HIPPT_CL BeginPlan begin_plan(unsigned c0, unsigned own, unsigned nfin, unsigned slots, unsigned cap) {
    BeginPlan b;
    b.t0 = begin_t0(c0, own);
    const int a = int(b.t0 + nfin) - 1, o = int(own) - 1;
    b.c1 = a > o ? a : o;  // every batch before the own one, and the marked run from t0
    const int u = int(c0) > b.c1 + 1 ? int(c0) : b.c1 + 1;
    b.u = unsigned(u);
    const unsigned ringEnd = c0 + slots - 1u, capEnd = b.u + cap - 1u;
    b.tLim = ringEnd < capEnd ? ringEnd : capEnd;
    return b;
}
// The first batch not combined once this launch's combines are done (written for the next launch).
HIPPT_CL unsigned begin_next_c0(unsigned c0, int c1) { return int(c0) > c1 + 1 ? c0 : unsigned(c1 + 1); }

// ---- a wave moving on (chain_next) -------------------------------------------------------------
// The batch after the wave's batch t (the own group, ChainWave::stat, is followed by the batch after
// the group).
HIPPT_CL unsigned next_batch(unsigned t, unsigned stat, unsigned group) { return t == stat ? t + group : t + 1u; }
// The frames of batch tItem from the launch's own batch's (chainSeq): its step times the distance.
HIPPT_CL unsigned frame_add(unsigned tItem, unsigned own, int step) {
    return (tItem - own) * unsigned(step > 0 ? step : 0);
}
// The group position -> (batch, one-batch position) split of a group launch's queues: 64-item block
// m >> 6 is block (m >> 6) / group of batch t + (m >> 6) % group.
HIPPT_CL void group_item(unsigned got, unsigned t, unsigned group, unsigned &raw, unsigned &tItem) {
    if (group <= 1u) {
        raw = got;
        tItem = t;
        return;
    }
    const unsigned blk = got >> 6, q = blk / group;
    raw = (q << 6) | (got & 63u);
    tItem = t + (blk - q * group);
}

}  // namespace chain
}  // namespace hippt
