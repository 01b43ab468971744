// Baseline-JPEG decode of grayscale frames on gfx950: the decode half of
// SpeedTrain.__getitem__'s `Image.open(img_path).convert('RGB')` (REV/datasets/speed.py:209-210),
// which the reference runs in DataLoader worker processes (REV/main.py:252-254) through Pillow's
// libjpeg-turbo.  SPEED frames are 8-bit grayscale; convert('RGB') replicates the plane, which
// spe_preprocess does when it reads a 1-channel frame.
//
// Pipeline (all on the device, no host round trip; one launch sequence per batch):
//   parse      one thread per image walks the markers (SOI, DQT, SOF0/1, DHT, DRI, SOS, APPn,
//              COM): quantisation table, canonical Huffman tables (libjpeg jdhuff.c's derived
//              table: a 9-bit lookup + maxcode / valoffset per code length), frame size, restart
//              interval.  Progressive, arithmetic-coded, 12-bit, multi-component or multi-scan
//              files get a non-zero status and a zero frame.
//   unstuff    one workgroup per image: drops the stuffed 0x00 after 0xFF, splits the
//              entropy-coded data at RSTn markers into byte-aligned segments (restart
//              intervals), stops at the terminating marker; then cuts every segment into
//              SUBBITS-bit subsequences.
//   huffman    (Weissenberger & Schmidt's self-synchronising parallel decode) each subsequence
//              is decoded speculatively from its first bit with an assumed block-start state;
//              a sync round re-decodes subsequence k from the exit state of k-1 in lockstep with
//              its own speculative decode until the two decoders meet (Huffman codes resynchronise
//              within a few codewords), which fixes its block count; a per-segment pass verifies
//              the chain and re-decodes a segment sequentially if it never synchronised.
//   blocks     exclusive scan of the per-subsequence block counts -> each subsequence's first
//              block; a second decode writes DC differences and AC coefficients (natural order)
//   dc         segmented scan of the DC differences (predictor reset at each restart)
//   idct       libjpeg's jpeg_idct_islow (jidctint.c: 13-bit constants, PASS1_BITS 2, the
//              post-IDCT range-limit table with its & 1023 wrap), one thread per 8x8 block
//
// Bit-exact against Pillow itself (tests/test_jpeg.py).
#include "spe_common.h"
#include "spe_kernels.h"
#include "../../include/spe.h"

#include <climits>
#include <cstddef>
#include <string>

int spe_fail(int code, const std::string& msg);

namespace {

constexpr int LUTB = 9;                 // fast Huffman lookup bits
constexpr int SUBBITS = 2048;           // subsequence length (bits)
constexpr int UNSTUFF_NT = 1024;
constexpr int SCAN_NT = 1024;

struct HuffTab {
  uint16_t lut[1 << LUTB];              // (len << 8) | symbol for codes of <= LUTB bits, 0 = longer
  int32_t maxcode[18];                  // largest code of each length, -1 if none; [17] sentinel
  int32_t valoff[17];                   // huffval index = code + valoff[len]
  uint8_t huffval[256];
};

struct JpegImg {
  int status;
  int H, W, bw, bh, nblocks;
  int restart;                          // restart interval in blocks (MCUs), 0 = none
  int nseg, nsub;
  int64_t ecs_off;                      // entropy-coded data start in the file
  int ulen;                             // unstuffed bytes
  uint16_t qt[64];                      // natural order
  HuffTab dc, ac;
};

struct Sub {                            // one subsequence of one segment
  int start, end;                       // bit range [start, end) in the unstuffed stream
  int seg, first;                       // segment id, 1 if the segment's first subsequence
  int ep, ez;                           // entry state (bit, coefficient index)
  int xp, xz;                           // exit state
  int cnt;                              // blocks completed between entry and exit
  int blkp;                             // exclusive prefix of cnt over the image's subsequences
  int blk;                              // block index (image-wide) at entry
};

struct JpegWs {                         // device workspace carve-up (byte offsets)
  size_t imgs, subs, segblk, segstart, segfirst, segbad, stream, coef;
  int max_sub, max_seg, stream_stride, max_tiles;
  size_t tiles;
  size_t total;
};

enum { ST_OK = 0, ST_UNSUPPORTED = 1, ST_CORRUPT = 2, ST_SIZE = 3, ST_CAPACITY = 4 };

__constant__ uint8_t c_zz2nat[80] = {   // zig-zag index -> natural index (+16 guard entries)
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13,
    6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31,
    39, 46, 53, 60, 61, 54, 47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

// ------------------------------------------------------------------------------ parse
SPE_DEV int rd16(const uint8_t* p) { return (p[0] << 8) | p[1]; }

SPE_DEV bool build_table(HuffTab& t, const uint8_t* bits, const uint8_t* vals, int nvals) {
  // libjpeg jpeg_make_d_derived_tbl: canonical codes in order of length
  for (int i = 0; i < (1 << LUTB); ++i) t.lut[i] = 0;
  for (int i = 0; i < nvals; ++i) t.huffval[i] = vals[i];
  int code = 0, p = 0;
  for (int l = 1; l <= 16; ++l) {
    const int n = bits[l - 1];
    if (n) {
      t.valoff[l] = p - code;
      for (int i = 0; i < n; ++i, ++p, ++code) {
        if (l <= LUTB) {
          const int lo = code << (LUTB - l), hi = (code + 1) << (LUTB - l);
          for (int e = lo; e < hi; ++e) t.lut[e] = (uint16_t)((l << 8) | vals[p]);
        }
      }
      t.maxcode[l] = code - 1;
    } else {
      t.maxcode[l] = -1;
      t.valoff[l] = 0;
    }
    if (code >= (1 << l)) return false;  // no all-ones code (jpeg_make_d_derived_tbl)
    code <<= 1;
  }
  t.maxcode[17] = 0x7fffffff;
  t.maxcode[0] = -1;
  t.valoff[0] = 0;
  return p == nvals;
}

__global__ void jpeg_parse_kernel(const uint8_t* __restrict__ data, const int64_t* __restrict__ offs,
                                  const int64_t* __restrict__ sizes, int B, int H, int W, int64_t max_bytes,
                                  JpegImg* __restrict__ imgs) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  JpegImg& im = imgs[b];
  const uint8_t* d = data + offs[b];
  const int64_t n = sizes[b];
  im.status = ST_CORRUPT;
  im.nseg = im.nsub = 0;
  im.restart = 0;
  im.ulen = 0;
  im.H = H; im.W = W; im.bw = (W + 7) / 8; im.bh = (H + 7) / 8; im.nblocks = im.bw * im.bh;
  if (n > max_bytes) { im.status = ST_CAPACITY; return; }   // the unstuffed stream slot holds max_bytes
  if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) return;
  // table slots: 4 DC + 4 AC + 4 quant; defined bits
  uint16_t qts[4][64];
  int qdef = 0, hdef = 0, comp_id = -1, comp_tq = 0, fH = 0, fW = 0;
  int64_t p = 2;
  // Huffman tables are built straight into the image record once SOS names the slots; keep the
  // raw DHT segments' offsets until then
  int64_t dht_at[8];
  for (int i = 0; i < 8; ++i) dht_at[i] = -1;
  while (p + 4 <= n) {
    if (d[p] != 0xFF) return;                      // markers must follow one another
    while (p < n && d[p] == 0xFF) ++p;             // fill bytes
    if (p >= n) return;
    const int m = d[p++];
    if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
    if (m == 0xD9) return;                          // EOI before SOS
    if (p + 2 > n) return;
    const int len = rd16(d + p);
    if (len < 2 || p + len > n) return;
    const uint8_t* s = d + p + 2;
    const int sl = len - 2;
    if (m == 0xC0 || m == 0xC1) {                   // baseline / extended sequential, Huffman
      if (sl < 6 || s[0] != 8) { im.status = ST_UNSUPPORTED; return; }
      fH = rd16(s + 1); fW = rd16(s + 3);
      const int nf = s[5];
      if (nf != 1 || sl < 6 + 3 * nf) { im.status = ST_UNSUPPORTED; return; }
      comp_id = s[6];
      comp_tq = s[8] & 3;
    } else if ((m >= 0xC2 && m <= 0xCB && m != 0xC4 && m != 0xC8) || (m >= 0xCD && m <= 0xCF)) {
      im.status = ST_UNSUPPORTED;                   // progressive / lossless / arithmetic
      return;
    } else if (m == 0xC4) {                         // DHT: one or more tables
      int q = 0;
      while (q + 17 <= sl) {
        const int tc = s[q] >> 4, th = s[q] & 15;
        if (tc > 1 || th > 3) return;
        int cnt = 0;
        for (int i = 0; i < 16; ++i) cnt += s[q + 1 + i];
        if (cnt > 256 || q + 17 + cnt > sl) return;
        dht_at[tc * 4 + th] = p + 2 + q;
        hdef |= 1 << (tc * 4 + th);
        q += 17 + cnt;
      }
    } else if (m == 0xDB) {                         // DQT
      int q = 0;
      while (q < sl) {
        const int pq = s[q] >> 4, tq = s[q] & 15;
        if (tq > 3 || q + 1 + 64 * (pq + 1) > sl) return;
        for (int i = 0; i < 64; ++i)
          qts[tq][c_zz2nat[i]] = pq ? (uint16_t)rd16(s + q + 1 + 2 * i) : s[q + 1 + i];
        qdef |= 1 << tq;
        q += 1 + 64 * (pq + 1);
      }
    } else if (m == 0xDD) {                         // DRI
      if (sl < 2) return;
      im.restart = rd16(s);
    } else if (m == 0xDA) {                         // SOS
      if (comp_id < 0) return;
      const int ns = s[0];
      if (ns != 1 || sl < 6) { im.status = ST_UNSUPPORTED; return; }
      if (s[1] != comp_id) return;
      const int td = s[2] >> 4, ta = s[2] & 15;
      if (s[3] != 0 || s[4] != 63 || s[5] != 0) { im.status = ST_UNSUPPORTED; return; }
      if (td > 3 || ta > 3 || !(hdef >> td & 1) || !(hdef >> (4 + ta) & 1) || !(qdef >> comp_tq & 1)) return;
      if (fH != H || fW != W) { im.status = ST_SIZE; return; }
      for (int i = 0; i < 64; ++i) im.qt[i] = qts[comp_tq][i];
      const uint8_t* hd = d + dht_at[td];
      const uint8_t* ha = d + dht_at[4 + ta];
      int cd = 0, ca = 0;
      for (int i = 0; i < 16; ++i) { cd += hd[1 + i]; ca += ha[1 + i]; }
      if (!build_table(im.dc, hd + 1, hd + 17, cd) || !build_table(im.ac, ha + 1, ha + 17, ca)) return;
      im.ecs_off = offs[b] + p + len;
      im.status = ST_OK;
      return;
    }
    p += len;
  }
}

// ------------------------------------------------------------------------------ unstuff
// Byte i of the entropy-coded data (relative to ecs_off, within [0, n)): kept as data, dropped,
// an RSTn (dropped; a segment boundary), or the terminating marker.
enum { B_KEEP = 0, B_DROP = 1, B_RST = 2, B_END = 3 };
SPE_DEV int byte_kind(uint8_t prev, uint8_t cur, uint8_t next, bool has_prev) {
  if (cur == 0xFF) {
    if (next == 0x00) return B_KEEP;                // stuffed data byte 0xFF
    if (next >= 0xD0 && next <= 0xD7) return B_RST;
    if (next == 0xFF) return B_DROP;                // fill byte before a marker
    return B_END;
  }
  if (has_prev && prev == 0xFF && (cur == 0x00 || (cur >= 0xD0 && cur <= 0xD7))) return B_DROP;
  return B_KEEP;
}

SPE_DEV int block_scan_excl(int v, int* sh, int& total) {   // SCAN/UNSTUFF_NT threads, exclusive
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nw = blockDim.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[wid] = x;
  __syncthreads();
  if (wid == 0) {
    int w = lane < nw ? sh[lane] : 0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(w, o, 64);
      if (lane >= o) w += y;
    }
    if (lane < nw) sh[lane] = w;
  }
  __syncthreads();
  const int base = wid ? sh[wid - 1] : 0;
  total = sh[nw - 1];
  __syncthreads();
  return base + x - v;
}

// Unstuffing runs over tiles of UNSTUFF_NT x 16 bytes, one workgroup per (tile, image): each
// thread classifies 16 consecutive bytes (coalesced across the wave).  Pass 1 counts the kept
// bytes and restart markers of every tile up to the tile's first terminating marker; a per-image
// scan over the tiles (up to the first tile holding a terminating marker) gives each tile's
// output offset; pass 2 re-classifies and writes.  Then the segments (restart intervals) are
// cut into subsequences.
constexpr int UTILE = UNSTUFF_NT * 16;

struct TileBytes {
  uint8_t v[18];                                    // bytes i0-1 .. i0+16
  int kind[16];
  int end;                                          // first terminating marker of this thread, or INT_MAX
};

SPE_DEV void classify(const uint8_t* d, int n, int i0, TileBytes& t) {
#pragma unroll
  for (int e = 0; e < 18; ++e) {
    const int i = i0 - 1 + e;
    t.v[e] = i < 0 ? (uint8_t)0 : (i < n ? d[i] : (uint8_t)0xD9);      // past the data: as if EOI
  }
  t.end = INT_MAX;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    t.kind[e] = byte_kind(t.v[e], t.v[e + 1], t.v[e + 2], i0 + e > 0);
    if (i0 + e >= n) t.kind[e] = B_END;
    if (t.kind[e] == B_END && t.end == INT_MAX) t.end = i0 + e;
  }
}

// pass 1: per tile (kept, restarts) before the tile's first terminating marker, and that marker
__global__ __launch_bounds__(UNSTUFF_NT) void jpeg_unstuff_count_kernel(const uint8_t* __restrict__ data,
                                                                          const int64_t* __restrict__ offs,
                                                                          const int64_t* __restrict__ sizes,
                                                                          const JpegImg* __restrict__ imgs,
                                                                          int* __restrict__ tiles, JpegWs ws) {
  __shared__ int sh[UNSTUFF_NT / 64];
  __shared__ int s_end;
  const int b = blockIdx.y, tile = blockIdx.x, tid = threadIdx.x;
  const JpegImg& im = imgs[b];
  if (im.status != ST_OK) return;
  const int n = (int)(offs[b] + sizes[b] - im.ecs_off);
  const int t0 = tile * UTILE;
  int* tl = tiles + ((size_t)b * ws.max_tiles + tile) * 3;
  if (t0 >= n) {
    if (tid == 0) { tl[0] = 0; tl[1] = 0; tl[2] = INT_MAX; }
    return;
  }
  TileBytes t;
  classify(data + im.ecs_off, n, t0 + tid * 16, t);
  if (tid == 0) s_end = INT_MAX;
  __syncthreads();
  if (t.end != INT_MAX) atomicMin(&s_end, t.end);
  __syncthreads();
  const int end = s_end, i0 = t0 + tid * 16;
  int k = 0, r = 0;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const bool live = i0 + e < end;
    k += live && t.kind[e] == B_KEEP;
    r += live && t.kind[e] == B_RST;
  }
  int tot;
  block_scan_excl(k | (r << 16), sh, tot);
  if (tid == 0) { tl[0] = tot & 0xffff; tl[1] = tot >> 16; tl[2] = end; }
}

// per image: tile offsets (exclusive scans up to the first tile with a terminating marker)
__global__ __launch_bounds__(64) void jpeg_unstuff_scan_kernel(const int64_t* __restrict__ offs,
                                                                 const int64_t* __restrict__ sizes, JpegImg* imgs,
                                                                 int* __restrict__ tiles, JpegWs ws) {
  const int b = blockIdx.x;
  JpegImg& im = imgs[b];
  if (im.status != ST_OK || threadIdx.x) return;
  const int n = (int)(offs[b] + sizes[b] - im.ecs_off);
  const int nt = (n + UTILE - 1) / UTILE;
  int* tl = tiles + (size_t)b * ws.max_tiles * 3;
  int kept = 0, rst = 0, last = nt - 1;
  for (int i = 0; i < nt; ++i) {
    const int k = tl[3 * i], r = tl[3 * i + 1], e = tl[3 * i + 2];
    tl[3 * i] = kept;
    tl[3 * i + 1] = rst;
    kept += k;
    rst += r;
    if (e != INT_MAX) { last = i; break; }
  }
  for (int i = last + 1; i < nt; ++i) tl[3 * i + 2] = -1;        // past the end: nothing to write
  im.ulen = kept;
  im.nseg = rst + 1;
  if (rst + 1 > ws.max_seg) im.status = ST_CAPACITY;
}

// pass 2: write the kept bytes and the restart positions (segment starts)
__global__ __launch_bounds__(UNSTUFF_NT) void jpeg_unstuff_write_kernel(const uint8_t* __restrict__ data,
                                                                          const int64_t* __restrict__ offs,
                                                                          const int64_t* __restrict__ sizes,
                                                                          const JpegImg* __restrict__ imgs,
                                                                          const int* __restrict__ tiles,
                                                                          int* __restrict__ segstart,
                                                                          uint8_t* __restrict__ streams, JpegWs ws) {
  __shared__ int sh[UNSTUFF_NT / 64];
  __shared__ int s_end;
  const int b = blockIdx.y, tile = blockIdx.x, tid = threadIdx.x;
  const JpegImg& im = imgs[b];
  if (im.status != ST_OK) return;
  const int n = (int)(offs[b] + sizes[b] - im.ecs_off);
  const int t0 = tile * UTILE;
  const int* tl = tiles + ((size_t)b * ws.max_tiles + tile) * 3;
  if (t0 >= n || tl[2] == -1) return;
  TileBytes t;
  classify(data + im.ecs_off, n, t0 + tid * 16, t);
  if (tid == 0) s_end = INT_MAX;
  __syncthreads();
  if (t.end != INT_MAX) atomicMin(&s_end, t.end);
  __syncthreads();
  const int end = s_end, i0 = t0 + tid * 16;
  int k = 0, r = 0;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const bool live = i0 + e < end;
    k += live && t.kind[e] == B_KEEP;
    r += live && t.kind[e] == B_RST;
  }
  int tot;
  const int ex = block_scan_excl(k | (r << 16), sh, tot);
  uint8_t* out = streams + (size_t)b * ws.stream_stride;
  int* sst = segstart + (size_t)b * (ws.max_seg + 1);
  int o = tl[0] + (ex & 0xffff), rr = tl[1] + (ex >> 16);
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const bool live = i0 + e < end;
    if (live && t.kind[e] == B_KEEP) out[o++] = t.v[e + 1];
    else if (live && t.kind[e] == B_RST) sst[1 + rr++] = o;
  }
}

// segments -> blocks and subsequences (one workgroup per image)
__global__ __launch_bounds__(UNSTUFF_NT) void jpeg_segments_kernel(JpegImg* imgs, Sub* __restrict__ subs,
                                                                     int* __restrict__ segblk, int* __restrict__ segstart,
                                                                     int* __restrict__ segfirst, int* __restrict__ segbad,
                                                                     uint8_t* __restrict__ streams, JpegWs ws) {
  __shared__ int sh[UNSTUFF_NT / 64];
  const int b = blockIdx.x, tid = threadIdx.x;
  JpegImg& im = imgs[b];
  if (im.status != ST_OK) return;                   // block-uniform
  const int nseg = im.nseg, kept = im.ulen;
  uint8_t* out = streams + (size_t)b * ws.stream_stride;
  int* sst = segstart + (size_t)b * (ws.max_seg + 1);
  // zero padding past the data: the Huffman reader peeks up to 8 bytes ahead
  if (tid < 16) out[kept + tid] = 0;
  if (tid == 0) {
    sst[0] = 0;
    sst[nseg] = kept;
  }
  __syncthreads();
  const int R = im.restart > 0 ? im.restart : im.nblocks;
  const bool corrupt = ((long long)nseg - 1) * R >= im.nblocks;   // more intervals than blocks
  int* sb = segblk + (size_t)b * (ws.max_seg + 1);
  int* sf = segfirst + (size_t)b * (ws.max_seg + 1);
  Sub* sbs = subs + (size_t)b * ws.max_sub;
  int sub_base = 0;
  for (int s0 = 0; s0 < nseg; s0 += UNSTUFF_NT) {
    const int s = s0 + tid;
    int ns = 0;
    if (s < nseg) ns = max(1, ((sst[s + 1] - sst[s]) * 8 + SUBBITS - 1) / SUBBITS);
    int stot;
    const int sb0 = block_scan_excl(ns, sh, stot);
    if (s < nseg) {
      sb[s] = min(s * R, im.nblocks);
      const int first = sub_base + sb0;
      sf[s] = first;
      segbad[(size_t)b * (ws.max_seg + 1) + s] = 0;
      const int bit0 = sst[s] * 8, bit1 = sst[s + 1] * 8;
      for (int j = 0; j < ns; ++j) {
        const int k = first + j;
        if (k >= ws.max_sub) break;
        Sub& u = sbs[k];
        u.start = bit0 + j * SUBBITS;
        u.end = j + 1 == ns ? bit1 : bit0 + (j + 1) * SUBBITS;
        u.seg = s;
        u.first = j == 0;
        u.ep = u.start;
        u.ez = 0;
      }
    }
    sub_base += stot;
  }
  __syncthreads();
  if (tid == 0) {
    sb[nseg] = im.nblocks;
    im.nsub = sub_base;
    if (sub_base > ws.max_sub) im.status = ST_CAPACITY;
    if (corrupt) im.status = ST_CORRUPT;
  }
}

// ------------------------------------------------------------------------------ Huffman
struct Dec {
  int p, z, blocks;
};

struct BitSrc {
  const uint8_t* s;                                 // 256-byte aligned, 16 bytes of zero padding
  SPE_DEV uint32_t peek32(int p) const {            // bits p .. p+31, MSB first: two aligned words
    const uint32_t* q = reinterpret_cast<const uint32_t*>(s) + (p >> 5);
    const uint64_t w = ((uint64_t)__builtin_bswap32(q[0]) << 32) | __builtin_bswap32(q[1]);
    return (uint32_t)(w >> (32 - (p & 31)));
  }
};

// the image's two Huffman tables, copied into LDS by the workgroup (every workgroup of the
// Huffman kernels decodes subsequences of one image)
struct Tabs {
  HuffTab dc, ac;
};
SPE_DEV const Tabs& load_tabs(const JpegImg& im, Tabs* sh) {
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&im.dc);
  uint32_t* dst = reinterpret_cast<uint32_t*>(sh);
  static_assert(sizeof(Tabs) % 4 == 0 && offsetof(JpegImg, ac) == offsetof(JpegImg, dc) + sizeof(HuffTab), "layout");
  for (int i = threadIdx.x; i < (int)(sizeof(Tabs) / 4); i += blockDim.x) dst[i] = src[i];
  __syncthreads();
  return *sh;
}

// decode one symbol: returns the symbol, advances p by its code length
SPE_DEV int huff_sym(const HuffTab& t, uint32_t pk, int& len) {
  const int e = t.lut[pk >> (32 - LUTB)];
  if (e) {
    len = e >> 8;
    return e & 255;
  }
  int l = LUTB + 1;
  int code = (int)(pk >> (32 - l));
  while (l <= 16 && code > t.maxcode[l]) {
    ++l;
    code = (int)(pk >> (32 - l));
  }
  if (l > 16) {                                     // invalid code: libjpeg returns 0 (corrupt data)
    len = 16;
    return 0;
  }
  len = l;
  return t.huffval[(code + t.valoff[l]) & 255];
}

SPE_DEV int extend(uint32_t v, int s) { return s == 0 ? 0 : (v < (1u << (s - 1)) ? (int)v - (1 << s) + 1 : (int)v); }

// one decode step (one symbol and its value bits); WRITE stores the coefficient at zig-zag
// position z into blk[natural index] (the thread's LDS block slot)
template <bool WRITE>
SPE_DEV void step(const HuffTab& dc, const HuffTab& ac, const BitSrc& bs, Dec& st, int16_t* blk) {
  const uint32_t pk = bs.peek32(st.p);
  int len;
  if (st.z == 0) {
    const int s = huff_sym(dc, pk, len) & 15;
    const uint32_t v = s ? (uint32_t)(((uint64_t)pk << len) & 0xffffffffu) >> (32 - s) : 0u;
    if (WRITE) blk[0] = (int16_t)extend(v, s);
    st.p += len + s;
    st.z = 1;
  } else {
    const int rs = huff_sym(ac, pk, len);
    const int r = rs >> 4, s = rs & 15;
    if (s) {
      const int z = st.z + r;
      const uint32_t v = (uint32_t)(((uint64_t)pk << len) & 0xffffffffu) >> (32 - s);
      // (z <= 78: libjpeg's natural-order table maps the overflow entries to 63)
      if (WRITE) blk[c_zz2nat[z]] = (int16_t)extend(v, s);
      st.z = z + 1;
      st.p += len + s;
    } else {
      st.z = r == 15 ? st.z + 16 : 64;              // ZRL / EOB
      st.p += len;
    }
  }
  if (st.z >= 64) {
    st.z = 0;
    ++st.blocks;
  }
}

// decode from `st` until p >= end
SPE_DEV void run_to_count(const HuffTab& dc, const HuffTab& ac, const BitSrc& bs, Dec& st, int end) {
  while (st.p < end) step<false>(dc, ac, bs, st, nullptr);
}

SPE_DEV const uint8_t* stream_of(const JpegWs& ws, uint8_t* streams, int b) { return streams + (size_t)b * ws.stream_stride; }

constexpr int HUFF_NT = 256;

// speculative decode of every subsequence from its entry (subsequence start, block start)
__global__ __launch_bounds__(HUFF_NT) void jpeg_huff_spec_kernel(const JpegImg* __restrict__ imgs, Sub* subs,
                                                                   uint8_t* streams, JpegWs ws) {
  __shared__ Tabs tabs;
  const int b = blockIdx.y, k = blockIdx.x * HUFF_NT + threadIdx.x;
  const JpegImg& im = imgs[b];
  if (im.status != ST_OK || blockIdx.x * HUFF_NT >= im.nsub) return;     // workgroup-uniform
  const Tabs& t = load_tabs(im, &tabs);
  if (k >= im.nsub) return;
  Sub& u = subs[(size_t)b * ws.max_sub + k];
  BitSrc bs{stream_of(ws, streams, b)};
  Dec st{u.ep, u.ez, 0};
  run_to_count(t.dc, t.ac, bs, st, u.end);
  u.xp = st.p;
  u.xz = st.z;
  u.cnt = st.blocks;
}

// sync round: subsequence k (not first in its segment) re-decoded from the exit of k-1, in
// lockstep with the decode from its current entry, until they meet
__global__ __launch_bounds__(HUFF_NT) void jpeg_huff_sync_kernel(const JpegImg* __restrict__ imgs, const Sub* __restrict__ in,
                                                                   Sub* __restrict__ out, uint8_t* streams, JpegWs ws) {
  __shared__ Tabs tabs;
  const int b = blockIdx.y, k = blockIdx.x * HUFF_NT + threadIdx.x;
  const JpegImg& im = imgs[b];
  if (im.status != ST_OK || blockIdx.x * HUFF_NT >= im.nsub) return;     // workgroup-uniform
  const Tabs& t = load_tabs(im, &tabs);
  if (k >= im.nsub) return;
  const Sub* ib = in + (size_t)b * ws.max_sub;
  Sub u = ib[k];
  if (!u.first) {
    const Sub& pv = ib[k - 1];
    if (pv.xp != u.ep || pv.xz != u.ez) {
      BitSrc bs{stream_of(ws, streams, b)};
      Dec a{u.ep, u.ez, 0}, c{pv.xp, pv.xz, 0};
      bool synced = false;
      while (c.p < u.end) {
        if (a.p < c.p && a.p < u.end) step<false>(t.dc, t.ac, bs, a, nullptr);
        else if (c.p < a.p || a.p >= u.end) step<false>(t.dc, t.ac, bs, c, nullptr);
        else if (a.z == c.z) { synced = true; break; }
        else { step<false>(t.dc, t.ac, bs, a, nullptr); step<false>(t.dc, t.ac, bs, c, nullptr); }
      }
      if (synced) {
        u.cnt = u.cnt - a.blocks + c.blocks;        // same path from the meeting point on
      } else {
        u.xp = c.p; u.xz = c.z; u.cnt = c.blocks;
      }
      u.ep = pv.xp;
      u.ez = pv.xz;
    }
  }
  out[(size_t)b * ws.max_sub + k] = u;
}

// verify every link of the entry/exit chain (one thread per subsequence) and flag the segments
// with a broken one: a subsequence that never synchronised within the sync rounds
__global__ __launch_bounds__(HUFF_NT) void jpeg_huff_check_kernel(const JpegImg* __restrict__ imgs,
                                                                    const Sub* __restrict__ subs, int* segbad, JpegWs ws) {
  const int b = blockIdx.y, k = blockIdx.x * HUFF_NT + threadIdx.x;
  const JpegImg& im = imgs[b];
  if (im.status != ST_OK || k >= im.nsub) return;
  const Sub* sb = subs + (size_t)b * ws.max_sub;
  if (!sb[k].first && (sb[k].ep != sb[k - 1].xp || sb[k].ez != sb[k - 1].xz))
    segbad[(size_t)b * (ws.max_seg + 1) + sb[k].seg] = 1;
}

// re-decode a flagged segment sequentially (one thread per segment)
__global__ __launch_bounds__(HUFF_NT) void jpeg_huff_fix_kernel(const JpegImg* __restrict__ imgs, Sub* subs,
                                                                  const int* __restrict__ segfirst,
                                                                  const int* __restrict__ segbad, uint8_t* streams,
                                                                  JpegWs ws) {
  const int b = blockIdx.y, sgi = blockIdx.x * HUFF_NT + threadIdx.x;
  const JpegImg& im = imgs[b];
  if (im.status != ST_OK || sgi >= im.nseg || !segbad[(size_t)b * (ws.max_seg + 1) + sgi]) return;
  Sub* sb = subs + (size_t)b * ws.max_sub;
  const int k0 = segfirst[(size_t)b * (ws.max_seg + 1) + sgi];
  const int k1 = sgi + 1 < im.nseg ? segfirst[(size_t)b * (ws.max_seg + 1) + sgi + 1] : im.nsub;
  BitSrc bs{stream_of(ws, streams, b)};
  Dec st{sb[k0].start, 0, 0};
  for (int i = k0; i < k1; ++i) {
    sb[i].ep = st.p;
    sb[i].ez = st.z;
    st.blocks = 0;
    run_to_count(im.dc, im.ac, bs, st, sb[i].end);
    sb[i].xp = st.p;
    sb[i].xz = st.z;
    sb[i].cnt = st.blocks;
  }
}

// block index at each subsequence entry: segment's first block + the counts before it
__global__ __launch_bounds__(SCAN_NT) void jpeg_blocks_kernel(const JpegImg* __restrict__ imgs, Sub* subs,
                                                                const int* __restrict__ segblk, JpegWs ws) {
  __shared__ int sh[SCAN_NT / 64];
  const int b = blockIdx.x, tid = threadIdx.x;
  const JpegImg& im = imgs[b];
  if (im.status != ST_OK) return;
  Sub* sb = subs + (size_t)b * ws.max_sub;
  // global exclusive prefix of the counts -> blk = P[k]; jpeg_blocks_fix_kernel then subtracts
  // P at the segment's first subsequence and adds the segment's first block
  int carry = 0;
  for (int k0 = 0; k0 < im.nsub; k0 += SCAN_NT) {
    const int k = k0 + tid;
    const int c = k < im.nsub ? sb[k].cnt : 0;
    int tot;
    const int e = block_scan_excl(c, sh, tot);
    if (k < im.nsub) sb[k].blkp = carry + e;
    carry += tot;
  }
}

// block index at each entry = the segment's first block + the counts of the segment's earlier
// subsequences (one thread per subsequence).  The last subsequence of every segment also checks
// that the segment's data completed all of its blocks: a truncated entropy-coded segment (short
// file, short restart interval) would otherwise leave blocks unwritten -- the coefficient buffer
// is never cleared -- so the image is marked corrupt (Pillow raises "image file is truncated")
__global__ __launch_bounds__(HUFF_NT) void jpeg_blocks_fix_kernel(JpegImg* __restrict__ imgs, Sub* subs,
                                                                    const int* __restrict__ segblk,
                                                                    const int* __restrict__ segfirst, JpegWs ws) {
  const int b = blockIdx.y, k = blockIdx.x * HUFF_NT + threadIdx.x;
  JpegImg& im = imgs[b];
  if (im.status != ST_OK || k >= im.nsub) return;
  Sub* sb = subs + (size_t)b * ws.max_sub;
  const int sg = sb[k].seg;
  const size_t so = (size_t)b * (ws.max_seg + 1) + sg;
  const int p0 = sb[segfirst[so]].blkp;
  sb[k].blk = sb[k].blkp - p0 + segblk[so];
  if (k + 1 == im.nsub || sb[k + 1].seg != sg) {
    const int decoded = sb[k].blkp + sb[k].cnt - p0;
    if (decoded < segblk[so + 1] - segblk[so]) im.status = ST_CORRUPT;
  }
}

// decode again from the true entries, writing DC differences and AC coefficients (natural
// order) of every block the subsequence owns: each block is assembled in the thread's LDS slot and
// stored as 8 16-byte pieces; the block in progress at entry (owned from zig-zag position
// entry z on) and at exit (owned up to exit z) are stored position by position, zeros included,
// so every coefficient is written exactly once and the buffer needs no clearing
constexpr int SLOT_LD = 72;                 // int16 per LDS slot row (16-byte aligned, padded)
__global__ __launch_bounds__(HUFF_NT) void jpeg_huff_write_kernel(const JpegImg* __restrict__ imgs,
                                                                    const Sub* __restrict__ subs,
                                                                    const int* __restrict__ segblk, uint8_t* streams,
                                                                    int16_t* __restrict__ coef, int64_t coef_stride, JpegWs ws) {
  __shared__ __attribute__((aligned(16))) int16_t slots[HUFF_NT * SLOT_LD];
  __shared__ Tabs tabs;
  const int b = blockIdx.y, k = blockIdx.x * HUFF_NT + threadIdx.x;
  const JpegImg& im = imgs[b];
  if (im.status != ST_OK || blockIdx.x * HUFF_NT >= im.nsub) return;     // workgroup-uniform
  const Tabs& t = load_tabs(im, &tabs);
  if (k >= im.nsub) return;
  const Sub& u = subs[(size_t)b * ws.max_sub + k];
  const int seg_end = segblk[(size_t)b * (ws.max_seg + 1) + u.seg + 1];
  const int maxblk = seg_end - u.blk;
  int16_t* my = slots + threadIdx.x * SLOT_LD;
  int16_t* cb = coef + (size_t)b * coef_stride;
  auto clear = [&]() {
#pragma unroll
    for (int i = 0; i < 8; ++i) *reinterpret_cast<u32x4*>(my + 8 * i) = u32x4{0, 0, 0, 0};
  };
  auto store_range = [&](int blk, int z0, int z1) {          // zig-zag positions [z0, z1)
    for (int z = z0; z < z1; ++z) cb[(size_t)blk * 64 + c_zz2nat[z]] = my[c_zz2nat[z]];
  };
  BitSrc bs{stream_of(ws, streams, b)};
  Dec st{u.ep, u.ez, 0};
  int zstart = st.z;
  clear();
  while (st.p < u.end && st.blocks < maxblk) {
    const int before = st.blocks;
    step<true>(t.dc, t.ac, bs, st, my);
    if (st.blocks != before) {                      // block u.blk + before completed
      const int blk = u.blk + before;
      if (zstart == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
          *reinterpret_cast<u32x4*>(cb + (size_t)blk * 64 + 8 * i) = *reinterpret_cast<const u32x4*>(my + 8 * i);
      } else {
        store_range(blk, zstart, 64);
      }
      clear();
      zstart = 0;
    }
  }
  if (st.z != 0 && st.blocks < maxblk) store_range(u.blk + st.blocks, zstart, st.z);
}

// DC: running sum of the differences, reset at every restart (segment): a segmented inclusive
// scan over the blocks, SCAN_NT blocks per chunk with the carry between chunks
__global__ __launch_bounds__(SCAN_NT) void jpeg_dc_kernel(const JpegImg* __restrict__ imgs, int16_t* __restrict__ coef,
                                                            int64_t coef_stride) {
  __shared__ int sv[SCAN_NT / 64], sf[SCAN_NT / 64], s_carry;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  constexpr int NW = SCAN_NT / 64;
  const JpegImg& im = imgs[b];
  if (im.status != ST_OK) return;
  int16_t* c = coef + (size_t)b * coef_stride;
  const int R = im.restart > 0 ? im.restart : im.nblocks;
  if (tid == 0) s_carry = 0;
  __syncthreads();
  for (int k0 = 0; k0 < im.nblocks; k0 += SCAN_NT) {
    const int k = k0 + tid;
    const bool in = k < im.nblocks;
    int x = in ? c[(size_t)k * 64] : 0;
    int f = in && (k % R == 0);                     // segment head
    // (a, fa) + (b, fb) = (fb ? b : a + b, fa | fb), combined left into right
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64), g = __shfl_up(f, o, 64);
      if (lane >= o) {
        if (!f) x += y;
        f |= g;
      }
    }
    if (lane == 63) { sv[wid] = x; sf[wid] = f; }
    __syncthreads();
    if (wid == 0) {
      int w = lane < NW ? sv[lane] : 0, wf = lane < NW ? sf[lane] : 0;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(w, o, 64), g = __shfl_up(wf, o, 64);
        if (lane >= o) {
          if (!wf) w += y;
          wf |= g;
        }
      }
      if (lane < NW) { sv[lane] = w; sf[lane] = wf; }
    }
    __syncthreads();
    const int carry = s_carry;
    // everything left of this wave: earlier waves of the chunk, then the carry of earlier chunks
    const int left = wid == 0 ? carry : (sf[wid - 1] ? sv[wid - 1] : sv[wid - 1] + carry);
    const int incl = f ? x : x + left;
    if (in) c[(size_t)k * 64] = (int16_t)incl;
    __syncthreads();
    if (tid == SCAN_NT - 1) s_carry = incl;
    __syncthreads();
  }
}

// jpeg_idct_islow (libjpeg jidctint.c), one thread per block, u8 output
#define ISLOW_FIX(name, v) constexpr int name = v
ISLOW_FIX(F0298, 2446); ISLOW_FIX(F0390, 3196); ISLOW_FIX(F0541, 4433); ISLOW_FIX(F0765, 6270);
ISLOW_FIX(F0899, 7373); ISLOW_FIX(F1175, 9633); ISLOW_FIX(F1501, 12299); ISLOW_FIX(F1847, 15137);
ISLOW_FIX(F1961, 16069); ISLOW_FIX(F2053, 16819); ISLOW_FIX(F2562, 20995); ISLOW_FIX(F3072, 25172);
constexpr int CONST_BITS = 13, PASS1_BITS = 2;

// 32-bit arithmetic: for coefficients an 8-bit encoder produces (dequantised |value| < 2^15)
// every intermediate fits, as in libjpeg-turbo's SIMD islow (16-bit dequantisation, 32-bit
// pmaddwd products), so the results equal jidctint.c's 64-bit JLONG ones
SPE_DEV int descale(int x, int n) { return (x + (1 << (n - 1))) >> n; }

// post-IDCT range limit: libjpeg's table indexed by (value & 1023) with CENTERJSAMPLE added
SPE_DEV uint8_t range_limit(int v) {
  const int i = v & 1023;
  if (i < 128) return (uint8_t)(i + 128);
  if (i < 512) return 255;
  if (i < 896) return 0;
  return (uint8_t)(i - 896);
}

SPE_DEV void idct_1d(int d0, int d1, int d2, int d3, int d4, int d5, int d6, int d7, int out[8]) {
  // even part
  int z2 = d2, z3 = d6;
  int z1 = (z2 + z3) * F0541;
  const int tmp2e = z1 + z3 * (-F1847);
  const int tmp3e = z1 + z2 * F0765;
  z2 = d0; z3 = d4;
  const int tmp0e = (z2 + z3) * (1 << CONST_BITS);
  const int tmp1e = (z2 - z3) * (1 << CONST_BITS);
  const int tmp10 = tmp0e + tmp3e, tmp13 = tmp0e - tmp3e, tmp11 = tmp1e + tmp2e, tmp12 = tmp1e - tmp2e;
  // odd part
  int tmp0 = d7, tmp1 = d5, tmp2 = d3, tmp3 = d1;
  z1 = tmp0 + tmp3;
  z2 = tmp1 + tmp2;
  z3 = tmp0 + tmp2;
  int z4 = tmp1 + tmp3;
  const int z5 = (z3 + z4) * F1175;
  tmp0 = tmp0 * F0298;
  tmp1 = tmp1 * F2053;
  tmp2 = tmp2 * F3072;
  tmp3 = tmp3 * F1501;
  z1 = z1 * (-F0899);
  z2 = z2 * (-F2562);
  z3 = z3 * (-F1961);
  z4 = z4 * (-F0390);
  z3 += z5;
  z4 += z5;
  tmp0 += z1 + z3;
  tmp1 += z2 + z4;
  tmp2 += z2 + z3;
  tmp3 += z1 + z4;
  out[0] = tmp10 + tmp3; out[7] = tmp10 - tmp3;
  out[1] = tmp11 + tmp2; out[6] = tmp11 - tmp2;
  out[2] = tmp12 + tmp1; out[5] = tmp12 - tmp1;
  out[3] = tmp13 + tmp0; out[4] = tmp13 - tmp0;
}

__global__ __launch_bounds__(256) void jpeg_idct_kernel(const JpegImg* __restrict__ imgs, const int16_t* __restrict__ coef,
                                                          int64_t coef_stride, uint8_t* __restrict__ frames, int H, int W,
                                                          int32_t* __restrict__ status) {
  const int b = blockIdx.y;
  const JpegImg& im = imgs[b];
  const int blk = blockIdx.x * blockDim.x + threadIdx.x;
  if (blk == 0 && status) status[b] = im.status;
  if (blk >= im.nblocks) return;
  const int by = blk / im.bw, bx = blk - by * im.bw;
  uint8_t* out = frames + (size_t)b * H * W;
  if (im.status != ST_OK) {                         // undecodable image: zero frame
    for (int r = 0; r < 8 && by * 8 + r < H; ++r)
      for (int c = 0; c < 8 && bx * 8 + c < W; ++c) out[(size_t)(by * 8 + r) * W + bx * 8 + c] = 0;
    return;
  }
  const int16_t* cb = coef + (size_t)b * coef_stride + (size_t)blk * 64;
  int ws[64];
  int q[64];
  {
    const int4* c4 = reinterpret_cast<const int4*>(cb);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int4 v = c4[i];
      const int w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        q[8 * i + 2 * e] = (int)(int16_t)(w[e] & 0xffff) * (int)im.qt[8 * i + 2 * e];
        q[8 * i + 2 * e + 1] = (int)(int16_t)((uint32_t)w[e] >> 16) * (int)im.qt[8 * i + 2 * e + 1];
      }
    }
  }
  // pass 1: columns
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    int o[8];
    idct_1d(q[c], q[8 + c], q[16 + c], q[24 + c], q[32 + c], q[40 + c], q[48 + c], q[56 + c], o);
#pragma unroll
    for (int r = 0; r < 8; ++r) ws[8 * r + c] = descale(o[r], CONST_BITS - PASS1_BITS);
  }
  // pass 2: rows
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    int o[8];
    const int* w = ws + 8 * r;
    idct_1d(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], o);
    const int y = by * 8 + r;
    if (y >= H) continue;
    uint8_t px[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) px[c] = range_limit(descale(o[c], CONST_BITS + PASS1_BITS + 3));
    uint8_t* row = out + (size_t)y * W + bx * 8;
    if (bx * 8 + 8 <= W && (W & 7) == 0) {
      uint32_t lo = px[0] | (px[1] << 8) | (px[2] << 16) | ((uint32_t)px[3] << 24);
      uint32_t hi = px[4] | (px[5] << 8) | (px[6] << 16) | ((uint32_t)px[7] << 24);
      *reinterpret_cast<uint2*>(row) = uint2{lo, hi};
    } else {
      for (int c = 0; c < 8 && bx * 8 + c < W; ++c) row[c] = px[c];
    }
  }
}

JpegWs plan(int B, int H, int W, int64_t max_bytes) {
  JpegWs w{};
  const int nblocks = ((H + 7) / 8) * ((W + 7) / 8);
  w.max_seg = nblocks + 1;
  w.max_sub = (int)((max_bytes * 8 + SUBBITS - 1) / SUBBITS) + w.max_seg + 1;
  w.stream_stride = (int)((max_bytes + 64 + 255) / 256 * 256);
  w.max_tiles = (int)((max_bytes + UTILE - 1) / UTILE);
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off += (bytes + 255) / 256 * 256; return o; };
  w.imgs = take(sizeof(JpegImg) * (size_t)B);
  w.subs = take(sizeof(Sub) * (size_t)B * w.max_sub * 2);     // two buffers for the sync rounds
  w.segblk = take(sizeof(int) * (size_t)B * (w.max_seg + 1));
  w.segstart = take(sizeof(int) * (size_t)B * (w.max_seg + 1));
  w.segfirst = take(sizeof(int) * (size_t)B * (w.max_seg + 1));
  w.segbad = take(sizeof(int) * (size_t)B * (w.max_seg + 1));
  w.tiles = take(sizeof(int) * 3 * (size_t)B * w.max_tiles);
  w.stream = take((size_t)B * w.stream_stride);
  w.coef = take((size_t)B * nblocks * 64 * 2);
  w.total = off;
  return w;
}

}  // namespace

extern "C" {

int64_t spe_jpeg_workspace_bytes(int batch, int height, int width, int64_t max_bytes_per_image) {
  if (batch < 0 || height <= 0 || width <= 0 || max_bytes_per_image <= 0) return -1;
  return (int64_t)plan(batch, height, width, max_bytes_per_image).total;
}

int spe_jpeg_decode(void* stream, const uint8_t* data, const int64_t* offsets, const int64_t* sizes, int batch,
                    int height, int width, int64_t max_bytes_per_image, uint8_t* frames, int32_t* status,
                    void* workspace, int64_t workspace_bytes) {
  if (!data || !offsets || !sizes || !frames || !workspace || batch < 0 || height <= 0 || width <= 0 ||
      height > 65535 || width > 65535 || max_bytes_per_image <= 0)
    return spe_fail(SPE_E_ARG, "bad argument");
  if (batch == 0) return 0;
  const JpegWs w = plan(batch, height, width, max_bytes_per_image);
  if ((int64_t)w.total > workspace_bytes) return spe_fail(SPE_E_WORKSPACE, "jpeg workspace too small");
  hipStream_t s = (hipStream_t)stream;
  char* base = (char*)workspace;
  JpegImg* imgs = (JpegImg*)(base + w.imgs);
  Sub* subs0 = (Sub*)(base + w.subs);
  Sub* subs1 = subs0 + (size_t)batch * w.max_sub;
  int* segblk = (int*)(base + w.segblk);
  int* segstart = (int*)(base + w.segstart);
  uint8_t* streams = (uint8_t*)(base + w.stream);
  int16_t* coef = (int16_t*)(base + w.coef);
  const int nblocks = ((height + 7) / 8) * ((width + 7) / 8);
  const int64_t cstride = (int64_t)nblocks * 64;
  hipLaunchKernelGGL(jpeg_parse_kernel, dim3((batch + 63) / 64), dim3(64), 0, s, data, offsets, sizes, batch, height,
                     width, max_bytes_per_image, imgs);
  int* segfirst = (int*)(base + w.segfirst);
  int* segbad = (int*)(base + w.segbad);
  int* tiles = (int*)(base + w.tiles);
  const dim3 gt(w.max_tiles, batch);
  hipLaunchKernelGGL(jpeg_unstuff_count_kernel, gt, dim3(UNSTUFF_NT), 0, s, data, offsets, sizes, imgs, tiles, w);
  hipLaunchKernelGGL(jpeg_unstuff_scan_kernel, dim3(batch), dim3(64), 0, s, offsets, sizes, imgs, tiles, w);
  hipLaunchKernelGGL(jpeg_unstuff_write_kernel, gt, dim3(UNSTUFF_NT), 0, s, data, offsets, sizes, imgs, tiles, segstart,
                     streams, w);
  hipLaunchKernelGGL(jpeg_segments_kernel, dim3(batch), dim3(UNSTUFF_NT), 0, s, imgs, subs0, segblk, segstart, segfirst,
                     segbad, streams, w);
  const dim3 sg((w.max_sub + HUFF_NT - 1) / HUFF_NT, batch);
  const dim3 gseg((w.max_seg + HUFF_NT - 1) / HUFF_NT, batch);
  hipLaunchKernelGGL(jpeg_huff_spec_kernel, sg, dim3(HUFF_NT), 0, s, imgs, subs0, streams, w);
  // two sync rounds (ping-pong), then the chain check and the sequential repair of any segment
  // that did not synchronise
  hipLaunchKernelGGL(jpeg_huff_sync_kernel, sg, dim3(HUFF_NT), 0, s, imgs, subs0, subs1, streams, w);
  hipLaunchKernelGGL(jpeg_huff_sync_kernel, sg, dim3(HUFF_NT), 0, s, imgs, subs1, subs0, streams, w);
  hipLaunchKernelGGL(jpeg_huff_check_kernel, sg, dim3(HUFF_NT), 0, s, imgs, subs0, segbad, w);
  hipLaunchKernelGGL(jpeg_huff_fix_kernel, gseg, dim3(HUFF_NT), 0, s, imgs, subs0, segfirst, segbad, streams, w);
  hipLaunchKernelGGL(jpeg_blocks_kernel, dim3(batch), dim3(SCAN_NT), 0, s, imgs, subs0, segblk, w);
  hipLaunchKernelGGL(jpeg_blocks_fix_kernel, sg, dim3(HUFF_NT), 0, s, imgs, subs0, segblk, segfirst, w);
  hipLaunchKernelGGL(jpeg_huff_write_kernel, sg, dim3(HUFF_NT), 0, s, imgs, subs0, segblk, streams, coef, cstride, w);
  hipLaunchKernelGGL(jpeg_dc_kernel, dim3(batch), dim3(SCAN_NT), 0, s, imgs, coef, cstride);
  hipLaunchKernelGGL(jpeg_idct_kernel, dim3((nblocks + 255) / 256, batch), dim3(256), 0, s, imgs, coef, cstride, frames,
                     height, width, status);
  const int e = (int)hipGetLastError();
  if (e) return spe_fail(e, "jpeg launch failed");
  return 0;
}

}  // extern "C"
