// p64gpu_abi.hip -- the C ABI of libp64gpu (include/p64gpu.h): argument
// validation, the choice of kernels per call, launch splitting for batches
// over 2 GiB, the ME-record scratch of the split inter encoder and the
// host-buffer encoder context.  The kernels live in k_search.hip (one wave
// per macroblock), k_block.hip (one lane per 8x8 block) and k_aux.hip.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/p64gpu.h"
#include "launch.h"
#include "vlc_count.h"

extern "C" int p64gpu_vlc_len_table_(uint32_t *out);
extern "C" const uint32_t *p64gpu_vlc_len_dev_(void *stream);
extern "C" int p64gpu_vlc_block_bits_(int width, int height, int nframes, const p64_mb_rec *mb,
                                      const int16_t *coef, uint16_t *blk_bits, void *stream);

namespace {

// ---------------------------------------------------------------------------
// error reporting

thread_local char g_err[512];

int fail(int status, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return status;
}

#define HIP_TRY(expr)                                                        \
  do {                                                                       \
    hipError_t e_ = (expr);                                                  \
    if (e_ != hipSuccess)                                                    \
      return fail(P64GPU_E_HIP, "%s: %s", #expr, hipGetErrorString(e_));     \
  } while (0)

// ---------------------------------------------------------------------------
// host-side validation

int check_geometry(int w, int h, int nframes, int64_t stride, bool luma_only = false) {
  if (w < 32 || h < 32 || w > 4096 || h > 4096 || (w & 15) || (h & 15))
    return fail(P64GPU_E_INVALID, "picture %dx%d: need multiples of 16 in 32..4096", w, h);
  if (nframes < 1) return fail(P64GPU_E_INVALID, "nframes %d < 1", nframes);
  const int64_t need = luma_only ? (int64_t)w * h : (int64_t)w * h * 3 / 2;
  if (stride < need || (stride & 15))
    return fail(P64GPU_E_INVALID, "frame_stride %lld: need >= %lld and a multiple of 16",
                (long long)stride, (long long)need);
  const int64_t blocks = (int64_t)nframes * (w / 16) * (h / 16);
  if (blocks >= (1LL << 30)) return fail(P64GPU_E_INVALID, "too many macroblocks in one call");
  return P64GPU_OK;
}

bool aligned(const void *p, uintptr_t n) { return ((uintptr_t)p & (n - 1)) == 0; }

// P64GPU_FUSED=1 (read once): intra and inter pictures through the fused
// one-wave-per-MB k_encode (the kernel of per-MB lists) instead of
// k_intra_mbg / k_motion + k_inter_mbg -- an A/B and cross-check switch,
// same results
bool fused_forced() {
  static const bool on = [] {
    const char *e = getenv("P64GPU_FUSED");
    return e && *e && *e != '0';
  }();
  return on;
}

// Device scratch for the ME records of the split inter encoder when the
// caller does not ask for them (args.me == NULL).
//  * One buffer per (device, stream), and per calling thread for
//    hipStreamPerThread (a sentinel that stands for each thread's own stream).
//  * The lock is held from the lookup until both kernels of the call are
//    enqueued, so calls from several threads on one shared stream (the NULL
//    stream, say) cannot interleave their k_motion / k_inter_mbg pairs: the
//    stream then orders them pair by pair.
//  * Never during stream capture: a captured graph would keep the buffer's
//    pointer and could race an eager call (or another graph replayed on
//    another stream) that uses it.  A capturing caller gets NULL and the
//    call takes the fused kernel, which needs no scratch.
//  * A buffer that is outgrown is retired, not freed (work still in flight
//    may reference it); p64gpu_release_scratch() frees everything when the
//    caller knows no such work remains.  The allocation runs in relaxed
//    capture mode, so it cannot invalidate another thread's global-mode
//    capture.
struct MeScratch {
  int dev;
  hipStream_t st;
  std::thread::id tid;
  p64_me_rec *buf;
  size_t cap;
};
std::mutex g_scr_mu;
std::vector<MeScratch> g_scr;
std::vector<void *> g_retired;

// returns the buffer with `lk` holding g_scr_mu, or NULL (lock not held)
p64_me_rec *me_scratch(size_t n, hipStream_t st, std::unique_lock<std::mutex> &lk) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  const std::thread::id tid = st == hipStreamPerThread ? std::this_thread::get_id() : std::thread::id();
  lk = std::unique_lock<std::mutex>(g_scr_mu);
  MeScratch *e = nullptr;
  for (auto &s : g_scr)
    if (s.dev == dev && s.st == st && s.tid == tid) e = &s;
  if (e && n <= e->cap) return e->buf;
  void *p = nullptr;
  hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
  (void)hipThreadExchangeStreamCaptureMode(&mode);
  const hipError_t me = hipMalloc(&p, n * sizeof(p64_me_rec));
  (void)hipThreadExchangeStreamCaptureMode(&mode);
  if (me != hipSuccess) {
    lk.unlock();
    return nullptr;
  }
  if (!e) {
    g_scr.push_back(MeScratch{dev, st, tid, nullptr, 0});
    e = &g_scr.back();
  }
  if (e->buf) g_retired.push_back(e->buf);
  e->buf = static_cast<p64_me_rec *>(p);
  e->cap = n;
  return e->buf;
}

}  // namespace

// the byte limit of one launch's buffers: the 2 GiB of a 32-bit buffer
// offset, or lower by P64GPU_CHUNK_BYTES (tests exercise the split launches
// with it); read on every call.  Also used by p64vlc.hip.
extern "C" int64_t p64gpu_chunk_bytes_(void) {
  int64_t lim = ((int64_t)1 << 31) - 1;
  const char *e = getenv("P64GPU_CHUNK_BYTES");
  if (e && *e) {
    const long long v = atoll(e);
    if (v > 0 && v < lim) lim = v;
  }
  return lim;
}

namespace {

// pictures per launch of the block-layout kernels: every buffer of a launch
// within p64gpu_chunk_bytes_() (per = the larger of a picture's bytes and its
// levels' bytes)
int pictures_per_launch(int w, int h, int64_t stride) {
  const int64_t levels = (int64_t)(w / 16) * (h / 16) * 768;
  const int64_t per = levels > stride ? levels : stride;
  const int64_t n = p64gpu_chunk_bytes_() / per;
  return n < 1 ? 1 : (int)n;
}

// pictures [f0, f0 + n) of a batch as a batch of its own
p64gpu_encode_args sub_batch(const p64gpu_encode_args &a, int f0, int n) {
  const size_t nmb = (size_t)(a.width / 16) * (a.height / 16), m0 = (size_t)f0 * nmb;
  p64gpu_encode_args c = a;
  c.nframes = n;
  c.cur = a.cur + (size_t)f0 * a.frame_stride;
  c.ref = a.ref ? a.ref + (size_t)f0 * a.frame_stride : nullptr;
  c.recon = a.recon + (size_t)f0 * a.frame_stride;
  c.last_intra = a.last_intra + m0;
  c.quant_mb = a.quant_mb ? a.quant_mb + m0 : nullptr;
  c.mtype_override = a.mtype_override ? a.mtype_override + m0 : nullptr;
  c.coef = a.coef + m0 * 384;
  c.mb = a.mb + m0;
  c.me = a.me ? a.me + m0 : nullptr;
  c.nzmask = a.nzmask ? a.nzmask + m0 : nullptr;
  c.vlc_bits = a.vlc_bits ? a.vlc_bits + m0 * 8 : nullptr;
  return c;
}

int encode_launch(const p64gpu_encode_args *a, const int32_t *mb_list, int count, void *stream) {
  if (!a) return fail(P64GPU_E_INVALID, "args is NULL");
  int s = check_geometry(a->width, a->height, a->nframes, a->frame_stride);
  if (s) return s;
  if (!a->cur || !a->recon || !a->last_intra || !a->coef || !a->mb)
    return fail(P64GPU_E_INVALID, "NULL required buffer");
  if (!a->intra && !a->ref) return fail(P64GPU_E_INVALID, "inter picture needs ref");
  if (!aligned(a->cur, 16) || !aligned(a->recon, 16) || !aligned(a->coef, 16) ||
      (!a->intra && !aligned(a->ref, 16)))
    return fail(P64GPU_E_INVALID, "cur/ref/recon/coef must be 16-byte aligned");
  if (!aligned(a->mb, 4) || (a->me && !aligned(a->me, 4)))
    return fail(P64GPU_E_INVALID, "mb/me records must be 4-byte aligned");
  if (a->quant < 1 || a->quant > 31) return fail(P64GPU_E_INVALID, "quant %d not in 1..31", a->quant);
  if (a->me_mode != P64GPU_ME_TSS && a->me_mode != P64GPU_ME_FULL)
    return fail(P64GPU_E_INVALID, "me mode %d", a->me_mode);
  if (a->search_limit < 1 || a->search_limit > 31)
    return fail(P64GPU_E_INVALID, "search_limit %d not in 1..31", a->search_limit);
  if (a->flags & ~(P64GPU_FLAG_ME_GIVEN | P64GPU_FLAG_SEARCH_ONLY))
    return fail(P64GPU_E_INVALID, "flags 0x%x: unknown bits", a->flags);
  if (a->vlc_bits && (mb_list || !aligned(a->vlc_bits, 16)))
    return fail(P64GPU_E_INVALID, "vlc_bits: 16-byte aligned, and not with an MB list");
  const uint32_t *vlc_len = nullptr;  // the count's code lengths, device copy (p64vlc.hip)
  if (a->vlc_bits && !(vlc_len = p64gpu_vlc_len_dev_(stream)))
    return fail(P64GPU_E_HIP, "vlc_bits: code-length table upload: %s", p64gpu_last_error());
  const bool me_given = (a->flags & P64GPU_FLAG_ME_GIVEN) != 0;
  if (me_given && (a->intra || !a->me || mb_list))
    return fail(P64GPU_E_INVALID, "P64GPU_FLAG_ME_GIVEN needs an inter picture batch with args->me");
  hipStream_t st = (hipStream_t)stream;
  const int mode = a->intra ? 0 : (a->me_mode == P64GPU_ME_FULL ? 2 : 1);
  if (a->flags & P64GPU_FLAG_SEARCH_ONLY) {  // the first half: the search into args->me
    if (me_given || a->intra || !a->me || mb_list)
      return fail(P64GPU_E_INVALID, "P64GPU_FLAG_SEARCH_ONLY needs an inter picture batch with args->me "
                                    "(and not ME_GIVEN)");
    HIP_TRY(p64k::motion(mode, a->width, a->height, a->nframes, a->frame_stride, a->ref, a->cur,
                         a->search_limit, a->me, /*stats: the ME_GIVEN half's*/ false, st));
    return P64GPU_OK;
  }
  if (!mb_list && (!fused_forced() || me_given)) {
    const int nmb = (a->width / 16) * (a->height / 16);
    // inter: ME for the whole batch into the caller's records or the scratch
    p64_me_rec *me = nullptr;
    std::unique_lock<std::mutex> lk;  // held while the scratch is in use (me_scratch)
    if (!a->intra) me = a->me ? a->me : me_scratch((size_t)a->nframes * nmb, st, lk);
    if (a->intra || me) {
      if (!a->intra && !me_given)
        HIP_TRY(p64k::motion(mode, a->width, a->height, a->nframes, a->frame_stride, a->ref, a->cur,
                             a->search_limit, me, /*stats: k_inter_mbg's*/ false, st));
      const int chunk = pictures_per_launch(a->width, a->height, a->frame_stride);
      for (int f0 = 0; f0 < a->nframes; f0 += chunk) {
        const p64gpu_encode_args c = sub_batch(*a, f0, a->nframes - f0 < chunk ? a->nframes - f0 : chunk);
        if (a->intra)
          HIP_TRY(p64k::intra_mbg(c, vlc_len, st));
        else
          HIP_TRY(p64k::inter_mbg(c, me + (size_t)f0 * nmb, vlc_len, st));
      }
      return P64GPU_OK;
    }
  }
  const unsigned grid =
      mb_list ? (unsigned)count : (unsigned)((int64_t)a->nframes * (a->width / 16) * (a->height / 16));
  HIP_TRY(p64k::encode_fused(mode, grid, *a, mb_list, st));
  if (a->vlc_bits)  // the fused kernel does not count: the entropy coder's count pass does
    return p64gpu_vlc_block_bits_(a->width, a->height, a->nframes, a->mb, a->coef, a->vlc_bits, stream);
  return P64GPU_OK;
}

}  // namespace

// ===========================================================================
// C ABI

extern "C" {

int p64gpu_abi_version(void) { return P64GPU_ABI_VERSION; }

const char *p64gpu_strerror(int s) {
  switch (s) {
    case P64GPU_OK: return "ok";
    case P64GPU_E_INVALID: return "invalid argument";
    case P64GPU_E_NODEVICE: return "no HIP device";
    case P64GPU_E_HIP: return "HIP runtime error";
    case P64GPU_E_NOMEM: return "out of memory";
    case P64GPU_E_STREAM: return "bitstream error";
    default: return "unknown status";
  }
}

const char *p64gpu_last_error(void) { return g_err; }

// error reporting for the host C parts of the library (p64stream.c)
int p64gpu_fail_(int status, const char *msg) { return fail(status, "%s", msg); }

int p64gpu_device_count(int *count) {
  if (!count) return fail(P64GPU_E_INVALID, "count is NULL");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  return P64GPU_OK;
}

int p64gpu_set_device(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
    return fail(P64GPU_E_NODEVICE, "no HIP device visible");
  if (device < 0 || device >= n) return fail(P64GPU_E_INVALID, "device %d of %d", device, n);
  HIP_TRY(hipSetDevice(device));
  return P64GPU_OK;
}

int p64gpu_synchronize(void *stream) {
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  return P64GPU_OK;
}

int p64gpu_alloc(void **ptr, size_t bytes) {
  if (!ptr) return fail(P64GPU_E_INVALID, "ptr is NULL");
  *ptr = nullptr;
  if (hipMalloc(ptr, bytes ? bytes : 1) != hipSuccess)
    return fail(P64GPU_E_NOMEM, "hipMalloc(%zu) failed", bytes);
  return P64GPU_OK;
}

int p64gpu_free(void *ptr) {
  if (ptr) HIP_TRY(hipFree(ptr));
  return P64GPU_OK;
}

int p64gpu_copy_to_device(void *dst, const void *src, size_t bytes, void *stream) {
  if ((!dst || !src) && bytes) return fail(P64GPU_E_INVALID, "NULL copy operand");
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
  return P64GPU_OK;
}

int p64gpu_copy_to_host(void *dst, const void *src, size_t bytes, void *stream) {
  if ((!dst || !src) && bytes) return fail(P64GPU_E_INVALID, "NULL copy operand");
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
  return P64GPU_OK;
}

int p64gpu_copy_on_device(void *dst, const void *src, size_t bytes, void *stream) {
  if ((!dst || !src) && bytes) return fail(P64GPU_E_INVALID, "NULL copy operand");
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return P64GPU_OK;
}

int p64gpu_block_op(int op, const int32_t *in, int32_t *out, int64_t nblocks, int dcq, int acq,
                    void *stream) {
  if (op < 0 || op >= P64GPU_OP_COUNT) return fail(P64GPU_E_INVALID, "block op %d", op);
  if (nblocks < 0) return fail(P64GPU_E_INVALID, "nblocks %lld", (long long)nblocks);
  if (nblocks == 0) return P64GPU_OK;
  if (!in || !out) return fail(P64GPU_E_INVALID, "NULL block buffer");
  const bool q = op >= P64GPU_OP_QUANT_INTRA && op <= P64GPU_OP_IQUANT_INTER;
  if (q && (dcq < 1 || acq < 1 || dcq > 255 || acq > 31))
    return fail(P64GPU_E_INVALID, "quantiser steps dcq=%d acq=%d", dcq, acq);
  if ((nblocks + 63) / 64 > 0x7fffffffLL) return fail(P64GPU_E_INVALID, "nblocks too large");
  HIP_TRY(p64k::block_op(op, in, out, nblocks, dcq, acq, (hipStream_t)stream));
  return P64GPU_OK;
}

int p64gpu_motion_estimation(int w, int h, int nframes, int64_t stride, const uint8_t *ref_y,
                             const uint8_t *cur_y, int mode, int sl, p64_me_rec *out,
                             void *stream) {
  int s = check_geometry(w, h, nframes, stride, true);
  if (s) return s;
  if (!ref_y || !cur_y || !out) return fail(P64GPU_E_INVALID, "NULL buffer");
  if (!aligned(ref_y, 16) || !aligned(cur_y, 16)) return fail(P64GPU_E_INVALID, "planes must be 16-byte aligned");
  if (!aligned(out, 4)) return fail(P64GPU_E_INVALID, "records must be 4-byte aligned");
  if (mode != P64GPU_ME_TSS && mode != P64GPU_ME_FULL) return fail(P64GPU_E_INVALID, "me mode %d", mode);
  if (sl < 1 || sl > 31) return fail(P64GPU_E_INVALID, "search_limit %d not in 1..31", sl);
  HIP_TRY(p64k::motion(mode == P64GPU_ME_FULL ? 2 : 1, w, h, nframes, stride, ref_y, cur_y, sl, out, true,
                       (hipStream_t)stream));
  return P64GPU_OK;
}

int p64gpu_encode_frames(const p64gpu_encode_args *a, void *stream) {
  return encode_launch(a, nullptr, 0, stream);
}

int p64gpu_encode_mb_list(const p64gpu_encode_args *a, const int32_t *mb_list, int count,
                          void *stream) {
  if (!a) return fail(P64GPU_E_INVALID, "args is NULL");
  if (a->nframes != 1) return fail(P64GPU_E_INVALID, "mb list needs nframes = 1");
  if (!mb_list || count < 0 || count > (a->width / 16) * (a->height / 16))
    return fail(P64GPU_E_INVALID, "mb list %p count %d", (const void *)mb_list, count);
  if (count == 0) return P64GPU_OK;
  return encode_launch(a, mb_list, count, stream);
}

int p64gpu_release_scratch(void) {
  std::lock_guard<std::mutex> lk(g_scr_mu);
  int dev0 = -1;
  (void)hipGetDevice(&dev0);
  for (auto &s : g_scr) {
    if (hipSetDevice(s.dev) == hipSuccess) (void)hipFree(s.buf);
  }
  for (void *p : g_retired) (void)hipFree(p);
  if (dev0 >= 0) (void)hipSetDevice(dev0);
  g_scr.clear();
  g_retired.clear();
  return P64GPU_OK;
}

int p64gpu_decode_recon(int w, int h, int nframes, int64_t stride, const uint8_t *ref,
                        uint8_t *recon, const int16_t *coef, const p64_mb_rec *mb,
                        const uint8_t *quant_mb, const uint8_t *coded_mask, void *stream) {
  int s = check_geometry(w, h, nframes, stride);
  if (s) return s;
  if (!ref || !recon || !coef || !mb || !quant_mb || !coded_mask)
    return fail(P64GPU_E_INVALID, "NULL buffer");
  if (!aligned(ref, 16) || !aligned(recon, 16) || !aligned(coef, 16) || !aligned(mb, 4))
    return fail(P64GPU_E_INVALID, "ref/recon/coef must be 16-byte aligned, mb 4-byte aligned");
  const size_t nmb = (size_t)(w / 16) * (h / 16);
  // pictures per launch: every buffer of a launch within the 2 GiB range of
  // the block kernels' 32-bit buffer offsets
  const int chunk = pictures_per_launch(w, h, stride);
  for (int f0 = 0; f0 < nframes; f0 += chunk) {
    const int nf = nframes - f0 < chunk ? nframes - f0 : chunk;
    const size_t m0 = (size_t)f0 * nmb;
    HIP_TRY(p64k::recon_mbg(w, h, nf, stride, ref + (size_t)f0 * stride, recon + (size_t)f0 * stride,
                            coef + m0 * 384, mb + m0, quant_mb + m0, coded_mask + m0, (hipStream_t)stream));
  }
  return P64GPU_OK;
}

int p64gpu_decode_recon_packed(int w, int h, int nframes, int64_t stride, const uint8_t *ref, uint8_t *recon,
                               const int16_t *levels, int64_t nlevels, const uint32_t *index,
                               const p64_mb_rec *mb, const uint8_t *quant_mb, const uint8_t *coded_mask,
                               void *stream) {
  int s = check_geometry(w, h, nframes, stride);
  if (s) return s;
  if (!ref || !recon || !index || !mb || !quant_mb || !coded_mask || (!levels && nlevels))
    return fail(P64GPU_E_INVALID, "NULL buffer");
  if (nlevels < 0 || nlevels >= (((int64_t)1) << 31) / 128)
    return fail(P64GPU_E_INVALID, "nlevels %lld: 0 .. 2^24-1 blocks per call", (long long)nlevels);
  if (!aligned(ref, 16) || !aligned(recon, 16) || !aligned(levels, 16) || !aligned(index, 16) || !aligned(mb, 4))
    return fail(P64GPU_E_INVALID, "ref/recon/levels/index must be 16-byte aligned, mb 4-byte aligned");
  const size_t nmb = (size_t)(w / 16) * (h / 16);
  // the index's groups run over the whole batch (64 blocks each, across
  // picture boundaries): a launch split starts on a group boundary, i.e. at a
  // multiple of 32 pictures (32 * 6 * nmb blocks = 3 * nmb groups)
  int chunk = pictures_per_launch(w, h, stride);
  if (chunk < nframes) {
    if (32 * stride >= ((int64_t)1 << 31)) return fail(P64GPU_E_INVALID, "decode_recon_packed: frame_stride");
    chunk = std::max(32, chunk & ~31);  // (32 pictures are always within range: 4096x4096 is ~805 MB)
  }
  for (int f0 = 0; f0 < nframes; f0 += chunk) {
    const int nf = nframes - f0 < chunk ? nframes - f0 : chunk;
    const size_t m0 = (size_t)f0 * nmb;
    HIP_TRY(p64k::recon_pk(w, h, nf, stride, ref + (size_t)f0 * stride, recon + (size_t)f0 * stride, levels,
                           (uint32_t)nlevels, index + m0 * 6 / 64 * 4, mb + m0, quant_mb + m0,
                           coded_mask + m0, (hipStream_t)stream));
  }
  return P64GPU_OK;
}

int p64gpu_synth_content(int content, int w, int h, uint32_t seed0, int nseeds, int frame0, int nslots,
                         int64_t stride, uint8_t *out, void *stream) {
  int s = check_geometry(w, h, 1, stride);
  if (s) return s;
  if (content != P64_SYNTH_VNOISE && content != P64_SYNTH_SURVEY)
    return fail(P64GPU_E_INVALID, "synth: content %d", content);
  if (!out || nseeds < 1 || nslots < 1 || frame0 < 0 || (int64_t)nseeds * nslots > 65535)
    return fail(P64GPU_E_INVALID, "synth: out=%p nseeds=%d nslots=%d frame0=%d", (void *)out,
                nseeds, nslots, frame0);
  HIP_TRY(p64k::synth(content, w, h, seed0, nseeds, frame0, nslots, stride, out, (hipStream_t)stream));
  return P64GPU_OK;
}

int p64gpu_synth_frames(int w, int h, uint32_t seed0, int nseeds, int frame0, int nslots,
                        int64_t stride, uint8_t *out, void *stream) {
  return p64gpu_synth_content(P64_SYNTH_VNOISE, w, h, seed0, nseeds, frame0, nslots, stride, out, stream);
}

int p64gpu_clock_probe(int microseconds, int *mhz, void *stream) {
  if (!mhz || microseconds < 1 || microseconds > 10000000)
    return fail(P64GPU_E_INVALID, "clock probe: mhz=%p microseconds=%d", (void *)mhz, microseconds);
  *mhz = 0;
  hipStream_t st = (hipStream_t)stream;
  const unsigned n = p64k::clock_waves();
  uint32_t *d = nullptr;
  HIP_TRY(hipMalloc(&d, (size_t)n * 2 * sizeof(uint32_t)));
  std::vector<uint32_t> h((size_t)n * 2);
  hipError_t e = p64k::clock((uint32_t)microseconds * 100u, d, st);  // 100 ticks per us
  if (e == hipSuccess) e = hipMemcpyAsync(h.data(), d, h.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(P64GPU_E_HIP, "clock probe: %s", hipGetErrorString(e));
  std::vector<double> f;
  for (unsigned i = 0; i < n; i++)
    if (h[2 * i + 1]) f.push_back(100.0 * h[2 * i] / h[2 * i + 1]);
  if (f.empty()) return fail(P64GPU_E_HIP, "clock probe: no samples");
  std::nth_element(f.begin(), f.begin() + f.size() / 2, f.end());
  *mhz = (int)(f[f.size() / 2] + 0.5);
  return P64GPU_OK;
}

// ---- host-buffer encoder context ------------------------------------------

struct p64gpu_encoder {
  int device, w, h, nmb, me_mode, sl;
  size_t pic;
  uint8_t *d_cur, *d_rec[2], *d_li;
  int8_t *d_ov;
  int16_t *d_coef;
  p64_mb_rec *d_mb;
  p64_me_rec *d_me;
  int cur_ref;  // index of the buffer holding the previous reconstruction
  hipStream_t stream;
};

static void enc_free(p64gpu_encoder *e) {
  if (!e) return;
  (void)hipFree(e->d_cur);
  (void)hipFree(e->d_rec[0]);
  (void)hipFree(e->d_rec[1]);
  (void)hipFree(e->d_li);
  (void)hipFree(e->d_ov);
  (void)hipFree(e->d_coef);
  (void)hipFree(e->d_mb);
  (void)hipFree(e->d_me);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  free(e);
}

int p64gpu_encoder_open(int device, int w, int h, int me_mode, int sl, p64gpu_encoder **out) {
  if (!out) return fail(P64GPU_E_INVALID, "out is NULL");
  *out = nullptr;
  int s = check_geometry(w, h, 1, (int64_t)w * h * 3 / 2);
  if (s) return s;
  if (me_mode != P64GPU_ME_TSS && me_mode != P64GPU_ME_FULL)
    return fail(P64GPU_E_INVALID, "me mode %d", me_mode);
  if (sl < 1 || sl > 31) return fail(P64GPU_E_INVALID, "search_limit %d", sl);
  s = p64gpu_set_device(device);
  if (s) return s;
  p64gpu_encoder *e = (p64gpu_encoder *)calloc(1, sizeof *e);
  if (!e) return fail(P64GPU_E_NOMEM, "host allocation");
  e->device = device;
  e->w = w;
  e->h = h;
  e->nmb = (w / 16) * (h / 16);
  e->me_mode = me_mode;
  e->sl = sl;
  e->pic = (size_t)w * h * 3 / 2;
  bool ok = hipMalloc(&e->d_cur, e->pic) == hipSuccess &&
            hipMalloc(&e->d_rec[0], e->pic) == hipSuccess &&
            hipMalloc(&e->d_rec[1], e->pic) == hipSuccess &&
            hipMalloc(&e->d_li, e->nmb) == hipSuccess &&
            hipMalloc(&e->d_ov, e->nmb) == hipSuccess &&
            hipMalloc(&e->d_coef, (size_t)e->nmb * 384 * sizeof(int16_t)) == hipSuccess &&
            hipMalloc(&e->d_mb, (size_t)e->nmb * sizeof(p64_mb_rec)) == hipSuccess &&
            hipMalloc(&e->d_me, (size_t)e->nmb * sizeof(p64_me_rec)) == hipSuccess &&
            hipStreamCreate(&e->stream) == hipSuccess;
  if (!ok) {
    enc_free(e);
    return fail(P64GPU_E_NOMEM, "device allocation for %dx%d encoder", w, h);
  }
  (void)hipMemset(e->d_rec[0], 0, e->pic);  // InitFS/ClearFS (p64.c:533-536)
  (void)hipMemset(e->d_rec[1], 0, e->pic);
  (void)hipMemset(e->d_li, 0, e->nmb);
  *out = e;
  return P64GPU_OK;
}

int p64gpu_encoder_frame(p64gpu_encoder *e, const uint8_t *picture, int intra, int quant,
                         const int8_t *mtype_override, int16_t *coef, p64_mb_rec *mb,
                         p64_me_rec *me, uint8_t *recon) {
  if (!e || !picture || !coef || !mb) return fail(P64GPU_E_INVALID, "NULL argument");
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipMemcpyAsync(e->d_cur, picture, e->pic, hipMemcpyHostToDevice, e->stream));
  if (intra) HIP_TRY(hipMemsetAsync(e->d_li, 0, e->nmb, e->stream));
  // the caller gets every block's levels: an inter picture writes only the
  // blocks with a nonzero level (include/p64gpu.h), the rest are zero
  if (!intra) HIP_TRY(hipMemsetAsync(e->d_coef, 0, (size_t)e->nmb * 384 * sizeof(int16_t), e->stream));
  if (mtype_override)
    HIP_TRY(hipMemcpyAsync(e->d_ov, mtype_override, e->nmb, hipMemcpyHostToDevice, e->stream));
  p64gpu_encode_args a;
  memset(&a, 0, sizeof a);
  a.width = e->w;
  a.height = e->h;
  a.nframes = 1;
  a.intra = intra ? 1 : 0;
  a.quant = quant;
  a.me_mode = e->me_mode;
  a.search_limit = e->sl;
  a.frame_stride = (int64_t)e->pic;
  a.cur = e->d_cur;
  a.ref = e->d_rec[e->cur_ref];
  a.recon = e->d_rec[e->cur_ref ^ 1];
  a.last_intra = e->d_li;
  a.mtype_override = mtype_override ? e->d_ov : nullptr;
  a.coef = e->d_coef;
  a.mb = e->d_mb;
  a.me = e->d_me;
  int s = p64gpu_encode_frames(&a, e->stream);
  if (s) return s;
  HIP_TRY(hipMemcpyAsync(coef, e->d_coef, (size_t)e->nmb * 384 * sizeof(int16_t),
                         hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipMemcpyAsync(mb, e->d_mb, (size_t)e->nmb * sizeof(p64_mb_rec), hipMemcpyDeviceToHost,
                         e->stream));
  if (me && !intra)
    HIP_TRY(hipMemcpyAsync(me, e->d_me, (size_t)e->nmb * sizeof(p64_me_rec),
                           hipMemcpyDeviceToHost, e->stream));
  if (recon)
    HIP_TRY(hipMemcpyAsync(recon, a.recon, e->pic, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  e->cur_ref ^= 1;  // SwapFS(CFS, OFS), p64.c:661
  return P64GPU_OK;
}

void p64gpu_encoder_close(p64gpu_encoder *e) { enc_free(e); }

}  // extern "C"
