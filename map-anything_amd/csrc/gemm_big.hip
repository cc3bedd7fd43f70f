// 256-row bf16 GEMM / implicit-GEMM convolution (gfx950): kernel choice and launch, the LayerNorm-fused residual
// linears, and the library's device fault word.  The kernel templates live in gemm_big_kernels.h and are instantiated
// in gemm_big_dense.hip / _conv / _f16 / _diag / _sk.hip (parallel build); see gemm_big_kernels.h for the design.
#include <atomic>

#include "gemm_big_kernels.h"

namespace mapa_gemm_impl {

// Sticky fault bits of the library (MAPA_FAULT_* in mapa.h), set by device code, read by mapa_fault_publish (into a
// host-visible slot, stream-ordered) and mapa_fault_status (synchronously).  Written with vector atomics only.  One
// word per calling host thread (FAULT_WORDS of them, 64 B apart; a thread's word is fixed at its first call): the
// per-call reset of one thread must not clear a fault another thread's concurrent call raised (two callers on two
// streams of one process — the in-thread sharded tests, a server with a model per stream).  One copy in this code
// object: kernels of the other translation units get the calling thread's word (GemmArgs.fault, fault_word()).
constexpr int FAULT_WORDS = 64, FAULT_STRIDE = 16;
__device__ unsigned g_mapa_fault[FAULT_WORDS * FAULT_STRIDE];

static int g_diag_grid = 0;  // mapa_gemm_tune(MAPA_TUNE_DIAG_GRID, .): timing diagnostic, 0 = the whole grid
void diag_set_grid(int blocks) { g_diag_grid = blocks; }

bool launch_gemm_big(const GemmArgs& a, bool conv, int variant, hipStream_t stream) {
  // variant: 0 = 256x256 / 128-B rows / 2 stages, 1 = 256x128 / 128 / 2, 2 = 256x256 / 64-B rows / 4 stages,
  //          3 = 256x128 / 64 / 4, 4 = 256x128 / 64 / 6, 5 = 256x128 / 128 / 3; 8 / 9 = 0 / 5 with s_setprio;
  //          10 / 11 = 256x128 / 64 / 3 at 2 per CU (11: s_setprio); 14 = 192x256, 15 = 192x192 (128-B rows, 2 stages);
  //          6, 7, 12, 13, 16..21: timing diagnostics and the ping-pong experiment (gemm_big_diag.hip)
  static const int bns[22] = {256, 128, 256, 128, 128, 128, 256, 256, 256, 128, 128, 128, 256, 256, 256, 192,
                              128, 128, 128, 256, 256, 256};
  static const int bms[22] = {256, 256, 256, 256, 256, 256, 256, 256, 256, 256, 256, 256, 256, 256, 192, 192,
                              256, 256, 256, 192, 192, 192};
  if (variant < 0 || variant > 21) return false;
  const int BN = bns[variant];
  const int BMv = bms[variant];
  int nblk = ((a.M + BMv - 1) / BMv) * ((a.N + BN - 1) / BN);
  const bool diag = variant == 6 || variant == 7 || variant == 12 || variant == 13 || variant >= 16;
  GemmKernel k = a.lp_f16 ? big_kernel_f16(variant, conv)
                 : diag   ? big_kernel_diag(variant, conv)
                 : conv   ? big_kernel_bf16_conv(variant)
                          : big_kernel_bf16_dense(variant);
  if (!k) return false;
  if (g_diag_grid > 0 && g_diag_grid < nblk) nblk = g_diag_grid;  // timing diagnostic: the first tiles only
  hipLaunchKernelGGL(k, dim3(nblk), dim3(BTHREADS), 0, stream, a);
  return true;
}


static int cur_device() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  return dev;
}

int gemm_device_cus() {  // CUs of the current device, cached per device (one process may drive several)
  static int cus_of[64] = {};
  const int dev = cur_device();
  int& cus = cus_of[dev];
  if (!cus) {
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  return cus;
}

// LayerNorm-fused residual linears: variant 14 = 192x256 tiles (N = 1024: the encoder's proj / fc2), 15 = 192x192
// (N = 768: the transformer's) — the shapes' data-parallel tiles, with the LNF epilogue and the band-major grid.
static int ln_bn(int variant) { return variant == 14 ? 256 : variant == 15 ? 192 : 0; }

int64_t ln_stats_bytes(int M, int N, int variant) {
  const int bn = ln_bn(variant);
  if (!bn || N % bn) return -1;
  return (int64_t)((M + 191) / 192) * LN_MAX_NTN * 192 * 16;  // 16-B granules, LN_MAX_NTN column-tile slots per band
}

static unsigned g_ln_spin = LN_SPIN_DEFAULT;  // mapa_gemm_tune(MAPA_TUNE_LN_SPIN, .)
static int g_ln_skip = 0;                      // mapa_gemm_tune(MAPA_TUNE_LN_TEST_SKIP, .): launches left to sabotage
void ln_set_spin(unsigned spins) { g_ln_spin = spins ? spins : LN_SPIN_DEFAULT; }
void ln_arm_test_skip(int n) { g_ln_skip = n; }
int ln_take_test_skip() {
  if (g_ln_skip <= 0) return 0;
  --g_ln_skip;
  return 1;
}
unsigned ln_spin_value() { return g_ln_spin; }
// DIAG (timing only, wrong results): MAPA_LN_DIAG 2 = no band wait, 4 = no LN stores, 8 = no f32 stores, 16 = no
// statistics / exchange at all (gemm_big LNF only)
int ln_diag_bits() {
  static int v = getenv("MAPA_LN_DIAG") ? (atoi(getenv("MAPA_LN_DIAG")) & 30) : 0;
  return v;
}


// Workgroups of an LNF kernel the current device holds at once (occupancy per CU x CUs), per device and variant.
static int lnf_slots(int variant, void (*k)(GemmArgs)) {
  static int slots[64][2] = {};
  int& s = slots[cur_device()][variant == 14 ? 0 : 1];
  if (!s) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, BTHREADS, 0) != hipSuccess || per_cu <= 0)
      per_cu = 1;
    s = per_cu * gemm_device_cus();
  }
  return s;
}

bool launch_gemm_big_ln(const GemmArgs& a, int variant, void* ws, int64_t ws_bytes, hipStream_t stream) {
  const int bn = ln_bn(variant);
  if (!bn || a.N % bn || a.lp_f16 || !a.ln_out || !a.ln_w || !a.ln_b || a.ln_ldo % 8 != 0) return false;
  // the in-place residual pattern (epi_mode 2): out_f32 = resid1 + gamma * (acc + bias), row-major, nothing else
  if (a.out_mode != 0 || !a.out_f32 || !a.resid1 || a.resid2 || a.out_lp || a.out_lp_relu || a.out_s3 ||
      a.out_s3_relu || a.act != MAPA_ACT_NONE || a.ldo % 8 != 0 || !a.vec_ok)
    return false;
  const int ntm = (a.M + 191) / 192, ntn = a.N / bn;
  if (ntn > LN_MAX_NTN || 2 * ntm >= LN_TICKET_WORDS || !ws || ws_bytes < GEMM_TICKET_BYTES + ln_stats_bytes(a.M, a.N, variant))
    return false;
  GemmKernel k = big_kernel_lnf(variant);
  // Co-residency by construction: every launch holds at most `slots` workgroups (lnf_grid rounds the bands up to a
  // multiple of the 8 XCDs), so a band's tiles never wait on a tile that cannot be dispatched until they finish.
  // Larger problems (batched scenes, the 100-view job) run as several launches of balanced band ranges.
  const int slots = lnf_slots(variant, k);
  const int nb_max = 8 * (slots / (8 * ntn));
  if (nb_max <= 0) return false;
  const int launches = (ntm + nb_max - 1) / nb_max;
  const int nb = (ntm + launches - 1) / launches;
  GemmArgs b = a;
  b.ln_ctr = reinterpret_cast<int*>(ws) + (GEMM_TICKET_BYTES / 4 - LN_TICKET_WORDS);
  b.ln_stats = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(ws) + GEMM_TICKET_BYTES);
  b.ln_spin = g_ln_spin;
  b.ln_skip = ln_diag_bits();
  if (g_ln_skip > 0) {
    b.ln_skip |= 1;
    --g_ln_skip;
  }
  for (int b0 = 0; b0 < ntm; b0 += nb) {
    b.ln_band0 = b0;
    b.ln_nbands = nb < ntm - b0 ? nb : ntm - b0;
    const int grid = mapa_idx::lnf_grid(b.ln_nbands, ntn);
    if (grid > slots) {  // cannot happen with nb <= nb_max; checked so a change to lnf_grid cannot break progress
      mapa_set_error("mapa_gemm: LayerNorm-fused launch of %d workgroups exceeds the %d co-resident slots", grid,
                     slots);
      return false;
    }
    hipLaunchKernelGGL(k, dim3(grid), dim3(BTHREADS), 0, stream, b);
    b.ln_skip &= ~1;
  }
  return true;
}

// The calling thread's fault word: stream-ordered reset and publish into a host-visible slot, synchronous read / reset.
__global__ void fault_reset_kernel(unsigned* word) {
  if (threadIdx.x == 0) __hip_atomic_store(word, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void fault_publish_kernel(const unsigned* word, unsigned* slot) {
  if (threadIdx.x == 0) {
    const unsigned f = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(slot, 1u | (f << 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static std::atomic<int> g_next_fault_word{0};

unsigned* fault_word() {
  static unsigned* base[16] = {nullptr};
  thread_local int word = -1;  // this host thread's word (threads past FAULT_WORDS share, round robin)
  if (word < 0) word = g_next_fault_word.fetch_add(1) % FAULT_WORDS;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) dev = 0;
  if (!base[dev]) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_mapa_fault)) == hipSuccess) base[dev] = static_cast<unsigned*>(p);
  }
  return base[dev] ? base[dev] + word * FAULT_STRIDE : nullptr;
}

}  // namespace mapa_gemm_impl


extern "C" int mapa_fault_slot_create(uint32_t** host, uint32_t** dev) {
  MAPA_CHECK_ARG(host && dev, "mapa_fault_slot_create: null output");
  void* h = nullptr;
  hipError_t e = hipHostMalloc(&h, 64, hipHostMallocCoherent | hipHostMallocMapped);
  if (e != hipSuccess) return mapa_set_error("mapa_fault_slot_create: hipHostMalloc: %s", hipGetErrorString(e));
  void* d = nullptr;
  e = hipHostGetDevicePointer(&d, h, 0);
  if (e != hipSuccess) {
    (void)hipHostFree(h);
    return mapa_set_error("mapa_fault_slot_create: hipHostGetDevicePointer: %s", hipGetErrorString(e));
  }
  memset(h, 0, 64);
  *host = static_cast<uint32_t*>(h);
  *dev = static_cast<uint32_t*>(d);
  return 0;
}

extern "C" int mapa_fault_slot_destroy(uint32_t* host) {
  if (!host) return 0;
  const hipError_t e = hipHostFree(host);
  return e == hipSuccess ? 0 : mapa_set_error("mapa_fault_slot_destroy: %s", hipGetErrorString(e));
}

extern "C" int mapa_fault_publish(uint32_t* dev_slot, hipStream_t stream) {
  MAPA_CHECK_ARG(dev_slot != nullptr, "mapa_fault_publish: null slot");
  unsigned* word = mapa_gemm_impl::fault_word();
  MAPA_CHECK_ARG(word != nullptr, "mapa_fault_publish: no fault word on this device");
  hipLaunchKernelGGL(mapa_gemm_impl::fault_publish_kernel, dim3(1), dim3(64), 0, stream, word,
                     reinterpret_cast<unsigned*>(dev_slot));
  MAPA_CHECK_LAUNCH("mapa_fault_publish");
  return 0;
}

extern "C" int mapa_fault_reset(hipStream_t stream) {
  unsigned* word = mapa_gemm_impl::fault_word();
  MAPA_CHECK_ARG(word != nullptr, "mapa_fault_reset: no fault word on this device");
  hipLaunchKernelGGL(mapa_gemm_impl::fault_reset_kernel, dim3(1), dim3(64), 0, stream, word);
  MAPA_CHECK_LAUNCH("mapa_fault_reset");
  return 0;
}

extern "C" int mapa_fault_status(int reset) {
  unsigned v = 0;
  unsigned* word = mapa_gemm_impl::fault_word();
  if (!word) {
    mapa_set_error("mapa_fault_status: no fault word on this device");
    return -1;
  }
  hipError_t e = hipMemcpy(&v, word, sizeof(v), hipMemcpyDeviceToHost);
  if (e != hipSuccess) {
    mapa_set_error("mapa_fault_status: %s", hipGetErrorString(e));
    return -1;
  }
  if (reset && v) {
    const unsigned zero = 0;
    e = hipMemcpy(word, &zero, sizeof(zero), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      mapa_set_error("mapa_fault_status: reset: %s", hipGetErrorString(e));
      return -1;
    }
  }
  return (int)v;
}
