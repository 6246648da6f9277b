// crc32c_list.hip -- the size-class list kernels (HCRC_SPLIT_SMALL) and the
// class-1 list kernel of the long-span split (HCRC_SPLIT_LONG): a partition
// pass sorts a batch into lists, each list runs one kernel.  These predate
// the lane-packed spans kernel (crc32c_lds.hip), which handles every span
// size in one launch; they stay as the opt-in flag paths of the C-ABI.
//
//   * run_ea: the end-aligned pipeline -- a span's segments END-aligned at
//     its last chunk, the first one partial (window chunks in front of it
//     zeroed), table blocks as a main segment + a front piece batched 16 per
//     iteration in 4-lane groups (crc32c_walk.h);
//   * run_g: G = 2 / 4 spans of at most 128 / 64 chunks per wave iteration,
//     one per group of 64 / G lanes, a start-aligned grid with ragged tails.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "crc32c_dev.h"
#include "crc32c_ea.h"
#include "crc32c_walk.h"

namespace wipdb {
namespace lk {

// ---------------------------------------------------------------------------
// Chunk geometry of the size-class lists' spans (run_g): a grid that starts
// at the span's first 16-byte-aligned chunk, with a ragged tail.
// ---------------------------------------------------------------------------
// The chunk geometry of a span at absolute address abs: h bytes of its first
// chunk lie in front of it, f full chunks, t tail bytes (for f == 0, the
// span's end inside chunk 0; 0 for an empty span).
struct Geo {
  uint32_t h, f, t;
  __device__ __forceinline__ Geo(uint64_t abs, uint32_t n) {
    h = static_cast<uint32_t>(abs & 15u);
    const uint32_t hn = h + n;
    f = hn >> 4;
    t = n == 0u ? 0u : (hn & 15u);
  }
};

// ---------------------------------------------------------------------------
// G = 2, 4: G spans per wave iteration, one per group of 64 / G lanes, each
// at most 256 / G chunks + a tail (a size-class list guarantees it).
// ---------------------------------------------------------------------------
template <int G>
struct GroupSpan {
  uint64_t a0;  // offset of the span's first chunk
  // full chunks (<= 256 / G) | head bytes << 8 | tail range [o, e) << 12, 16 |
  // valid << 24 -- packed: the G-span loop is short of SGPRs
  uint32_t pk;
  uint32_t init;
  uint32_t id;
  __device__ __forceinline__ uint32_t nc() const { return pk & 0xffu; }
  __device__ __forceinline__ uint32_t h() const { return (pk >> 8) & 15u; }
  __device__ __forceinline__ uint32_t o() const { return (pk >> 12) & 15u; }
  __device__ __forceinline__ uint32_t e() const { return (pk >> 16) & 31u; }
  __device__ __forceinline__ bool valid() const { return (pk >> 24) != 0u; }
};

template <int G, int OUT>
__device__ __forceinline__ void run_g(const ListSrc& src, void* out, uint32_t flags,
                                      const uint8_t* image) {
  constexpr uint32_t LG = 64u / G, CAP = kSegChunks / G;
  const uint32_t l = threadIdx.x & 63u;
  const uint32_t w = uni(threadIdx.x >> 6);
  const uint64_t count = src.count;
  if (static_cast<uint64_t>(blockIdx.x) * 16u >= count) return;
  load_image(image, w, l);
  const Lane lk = make_lane<G>(l);
  Pipe pp;
  pp.init(l, w);
  const bool msk = (flags & kFlagMask) != 0u;
  const uint64_t sbase = reinterpret_cast<uint64_t>(src.base);
  const uint32_t gl = l % LG;

  typedef GroupSpan<G> GS;
  // descriptors of the next G units (SMEM, waited for at first use)
  struct Pref {
    SpanD d[G];
    uint32_t nv;  // groups with a span (the first nv)
  };
  auto prefetch = [&](Pref& p) {
    const uint64_t s0 = grab_units<G>(l);
    p.nv = s0 >= count ? 0u : static_cast<uint32_t>(count - s0 < G ? count - s0 : G);
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (static_cast<uint32_t>(g) < p.nv) p.d[g] = src.get(s0 + g);
  };
  auto take = [&](const Pref& p, GS (&gs)[G]) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      gs[g].pk = gs[g].init = gs[g].id = 0;
      gs[g].a0 = 0;
      if (static_cast<uint32_t>(g) >= p.nv) continue;
      const SpanD& d = p.d[g];
      const Geo geo(sbase + d.a, d.n);
      gs[g].a0 = d.a - geo.h;
      gs[g].pk = geo.f | (geo.h << 8) | ((geo.f == 0u ? geo.h : 0u) << 12) | (geo.t << 16) |
                 (1u << 24);
      gs[g].init = d.init;
      gs[g].id = static_cast<uint32_t>(d.id);
    }
  };
  auto issue = [&](const GS (&gs)[G]) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (!gs[g].valid()) continue;
      if (gs[g].nc() != 0u) {
        if constexpr (G == 2) pp.issue<2>(sbase + gs[g].a0, 2u * g, CAP, gs[g].nc());
        else pp.issue<1>(sbase + gs[g].a0, static_cast<uint32_t>(g), CAP, gs[g].nc());
      }
      pp.issue_end(sbase + gs[g].a0 + 16u * gs[g].nc(), static_cast<uint32_t>(g),
                   gs[g].e() > gs[g].o(), OUT == 1, gs[g].e());
    }
  };
  // per-lane value of this lane's group: masked selects on per-group lane
  // masks (an opaque lane id keeps the compiler from turning the select
  // chain into an indexed scratch array -- scratch accesses would count in
  // vmcnt and break the hand-counted DMA waits)
  uint32_t lo = l;
  asm volatile("" : "+v"(lo));
  uint32_t gm[G];
#pragma unroll
  for (int g = 0; g < G; ++g) gm[g] = 0u - static_cast<uint32_t>(lo / LG == static_cast<uint32_t>(g));
  auto pick = [&](const uint32_t (&v)[G]) -> uint32_t {
    uint32_t r = v[0] & gm[0];
#pragma unroll
    for (int g = 1; g < G; ++g) r |= v[g] & gm[g];
    return r;
  };

  Pref pf;
  GS cur[G], nxt[G];
  prefetch(pf);
  if (pf.nv == 0u) return;
  take(pf, cur);
  prefetch(pf);
  issue(cur);
  bool stored_prev = false;

  for (;;) {
    if (stored_prev) wait_vm<1>();
    else wait_vm<0>();
    uint32_t W[16];
    pp.read(W);
    u32x4 tail[G], next[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      tail[g] = pp.piece(kAuxTail + g);
      next[g] = OUT == 1 ? pp.piece(kAuxNext + g) : u32x4{0, 0, 0, 0};
    }
    pp.release();
    const bool more = pf.nv != 0u;
    if (more) {
      take(pf, nxt);
      issue(nxt);
    }

    // ---- the G spans of this iteration ----
    uint32_t inj_g[G], nc_g[G], h_g[G];
    bool fast = true;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      inj_g[g] = cur[g].valid() ? head_register(l, cur[g].init, cur[g].h()) : 0u;
      nc_g[g] = cur[g].valid() ? cur[g].nc() : 0u;
      h_g[g] = cur[g].h();
      fast = fast && nc_g[g] == CAP && h_g[g] == 0u;
    }
    const uint32_t inj = pick(inj_g);
    if (fast) {
      W[0] ^= gl == 0u ? inj : 0u;
    } else {
      const int32_t base = static_cast<int32_t>(CAP - pick(nc_g));
      const uint32_t hh = pick(h_g);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int32_t ci = static_cast<int32_t>(4u * gl) + i - base;
#pragma unroll
        for (uint32_t ww = 0; ww < 4; ++ww)
          W[4 * i + ww] &= ci < 0 ? 0u : (ci == 0 ? head_mask(hh, ww) : ~0u);
        W[4 * i] ^= ci == 0 ? inj : 0u;
      }
    }
    const auto Rg = fold<G>(lk, l, scan(lk, W));
    // registers after the main chunks; all-tail spans start from ~init
    uint32_t R[G], o_g[G], e_g[G], tw[4][G], nw[4][G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      R[g] = cur[g].nc() == 0u ? ~cur[g].init : Rg[g];
      o_g[g] = cur[g].o();
      e_g[g] = cur[g].valid() ? cur[g].e() : 0u;
      tw[0][g] = tail[g].x;
      tw[1][g] = tail[g].y;
      tw[2][g] = tail[g].z;
      tw[3][g] = tail[g].w;
      nw[0][g] = next[g].x;
      nw[1][g] = next[g].y;
      nw[2][g] = next[g].z;
      nw[3][g] = next[g].w;
    }
    // tails, all groups in the same instructions (lane l serves its group;
    // the aux pieces were read by every lane, so the words are uniform per
    // group already)
    uint32_t r = pick(R);
    const uint32_t o = pick(o_g), e = pick(e_g);
    const u32x4 t{pick(tw[0]), pick(tw[1]), pick(tw[2]), pick(tw[3])};
    {
      uint32_t need = 0;
#pragma unroll
      for (int g = 0; g < G; ++g) need |= e_g[g];
      if (need != 0u) r = feed_tail_lanes(lk, l, r, t, o, e);
    }
    const uint32_t val = ~r;
    bool valid_l = false;
    uint32_t ids[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      ids[g] = cur[g].id;
      valid_l = valid_l || (gm[g] != 0u && cur[g].valid());
    }
    const uint32_t myid = pick(ids);
    if (gl == 0u && valid_l) {
      if (OUT == 1) {
        const u32x4 nx{pick(nw[0]), pick(nw[1]), pick(nw[2]), pick(nw[3])};
        static_cast<uint8_t*>(out)[myid] = unmask_crc(le32_at(t, nx, e)) == val ? 1u : 0u;
      } else {
        static_cast<uint32_t*>(out)[myid] = msk ? mask_crc(val) : val;
      }
    }
    stored_prev = true;

    if (!more) break;
#pragma unroll
    for (int g = 0; g < G; ++g) cur[g] = nxt[g];
    prefetch(pf);
  }
}

// A size-class list (HCRC_SPLIT_SMALL): G = 1 takes the spans of more than
// 128 chunks on the end-aligned pipeline (table blocks as main segment +
// front piece), G = 2 / 4 the spans of at most 128 / 64 chunks, several per
// wave iteration.  OUT: 0 = CRCs into out (u32, masked with kFlagMask),
// 1 = verify statuses into out (u8; the list lengths include the type byte).
template <int G, int OUT>
__global__ __launch_bounds__(kThreads) void crc32c_lds_list_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ len, const uint32_t* __restrict__ init,
    const uint32_t* __restrict__ id, const uint32_t* __restrict__ count, void* out,
    uint32_t flags, const uint8_t* __restrict__ image) {
  const ListSrc src{base, off, len, init, id, *count};
  if constexpr (G == 1) run_ea<OUT>(src, out, flags, image);
  else run_g<G, OUT>(src, out, flags, image);
}
#define WIPDB_LIST_KERNEL(G, OUT)                                                          \
  template __global__ void crc32c_lds_list_kernel<G, OUT>(                                 \
      const uint8_t*, const uint64_t*, const uint32_t*, const uint32_t*, const uint32_t*, \
      const uint32_t*, void*, uint32_t, const uint8_t*)
WIPDB_LIST_KERNEL(1, 0);
WIPDB_LIST_KERNEL(2, 0);
WIPDB_LIST_KERNEL(4, 0);
WIPDB_LIST_KERNEL(1, 1);
WIPDB_LIST_KERNEL(2, 1);
WIPDB_LIST_KERNEL(4, 1);
#undef WIPDB_LIST_KERNEL

// ---------------------------------------------------------------------------
// Partition into size-class lists (HCRC_SPLIT_SMALL).  Workgroup w scans a
// contiguous range of the batch twice: counts per class, one global atomic
// per class to reserve its slices, then writes the entries (wave-ordered
// through a ballot prefix), so each list keeps the batch's memory order
// piecewise.
// ---------------------------------------------------------------------------
constexpr int kPartThreads = 256;

// The class of a span of n bytes at address base + off: f = (a % 16 + n) / 16
// full chunks of its 16-byte grid; class 4: f <= 64, class 2: f <= 128,
// class 1: the rest.
__device__ __forceinline__ int class_slot(const uint8_t* base, uint64_t off, uint32_t n) {
  const uint32_t h = static_cast<uint32_t>((reinterpret_cast<uint64_t>(base) + off) & 15u);
  const uint32_t f = (h + n) >> 4;
  return f <= kClass4Chunks ? 2 : (f <= kClass2Chunks ? 1 : 0);
}

__global__ __launch_bounds__(kPartThreads) void crc32c_lds_partition_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ offsets,
    const uint32_t* __restrict__ lengths, const uint32_t* __restrict__ inits, uint64_t count,
    uint32_t extra, SpanList l1, SpanList l2, SpanList l4) {
  __shared__ uint32_t cnt[3], pos[3];
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint64_t per = (count + gridDim.x - 1) / gridDim.x;
  const uint64_t lo = per * blockIdx.x;
  const uint64_t hi = lo + per < count ? lo + per : count;
  if (tid < 3) cnt[tid] = 0;
  __syncthreads();
  // pass 1: count
  uint32_t mine[3] = {0, 0, 0};
  for (uint64_t s = lo + tid; s < hi; s += kPartThreads)
    ++mine[class_slot(base, offsets[s], lengths[s] + extra)];
#pragma unroll
  for (int k = 0; k < 3; ++k)
    if (mine[k]) atomicAdd(&cnt[k], mine[k]);
  __syncthreads();
  if (tid == 0) {
    pos[0] = cnt[0] ? atomicAdd(l1.count, cnt[0]) : 0u;
    pos[1] = cnt[1] ? atomicAdd(l2.count, cnt[1]) : 0u;
    pos[2] = cnt[2] ? atomicAdd(l4.count, cnt[2]) : 0u;
  }
  __syncthreads();
  // pass 2: positions (ballot prefix per wave step of 64 spans), then writes
  const uint64_t wbase = lo + (tid & ~63u);
  const uint64_t below = (uint64_t(1) << lane) - 1u;
  for (uint64_t s0 = wbase; s0 < hi; s0 += kPartThreads) {
    const uint64_t s = s0 + lane;
    const bool live = s < hi;
    uint64_t off = 0;
    uint32_t n = 0, ini = 0;
    int cls = -1;
    if (live) {
      off = offsets[s];
      n = lengths[s] + extra;
      ini = inits ? inits[s] : 0u;
      cls = class_slot(base, off, n);
    }
    uint32_t pa = 0;  // this lane's entry position
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const uint64_t m = __builtin_amdgcn_ballot_w64(cls == k);
      if (m == 0u) continue;
      uint32_t p0 = 0;
      if (lane == 0u) p0 = atomicAdd(&pos[k], static_cast<uint32_t>(__builtin_popcountll(m)));
      p0 = __builtin_amdgcn_readfirstlane(p0);
      if (cls == k) pa = p0 + __builtin_popcountll(m & below);
    }
    if (live) {
      const SpanList& L = cls == 0 ? l1 : (cls == 1 ? l2 : l4);
      L.off[pa] = off;
      L.len[pa] = n;
      L.init[pa] = ini;
      L.id[pa] = static_cast<uint32_t>(s);
    }
  }
}

}  // namespace lk
}  // namespace wipdb
