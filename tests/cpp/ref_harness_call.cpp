// The reference side of the boundary, compiled and run: a C++ program that
// declares the reference's registry FuncType exactly as mxmoe/kernels/src/include/registry.cuh:28-39
// does (half**, dim3*, mxmoe::QParams* — restated here, the reference headers need cutlass / fmt /
// thrust), registers the library's groupgemm_mxmoe in a registry-like table the way INTEGRATION.md
// §2 shows, builds the device / host arrays the way the reference harness does (one buffer per
// operand with running offsets, scale_zp = [sa(M) | sb(N)] per problem: test.cu:488-554) and calls
// the kernel through the function pointer as test.cu:793-813 does.
//
// This file deliberately does NOT include include/mxmoe_gg.h: a reference translation unit sees
// only its own types. tests/cpp/layout_check.cpp (linked into the same program) includes both
// sides' definitions and static_asserts that the layouts agree.
//
//   ref_harness_call --layout                 (no GPU: print the reference-side layouts)
//   ref_harness_call <in.bin> <out.bin>       (GPU: run the registered kernel on the problems in in.bin)
// in.bin: int32 P, then per problem int32 {M, N, K, a_bits, w_bits, gsize, sym}, then per problem the
// bytes of A, B (packed pack_wxax codes or fp16), sa (M fp16, quantised only), sb (N fp16, quantised only).
// out.bin: per problem C (M x N fp16, row-major, ldc = N).
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace mxmoe {
// quantize.cuh:14-25
struct QParams {
  int2 qbits{make_int2(16, 16)};
  int gsize{-1};
  bool sym{false};

  QParams() {}
  QParams(int2 _qbits, int _gsize, bool _sym) : qbits(_qbits), gsize(_gsize), sym(_sym) {}
};

// registry.cuh:28-39
using FuncType = void (*)(half** ptr_As, half** ptr_Bs, half** ptr_scale_a, half** ptr_scale_b, half** ptr_Cs,
                          half** ptr_Ds, int64_t* ldas, int64_t* ldbs, int64_t* ldcs, int64_t* ldds,
                          dim3* device_problem_sizes, dim3* host_problem_sizes, QParams* device_qbits_list,
                          QParams* host_qbits_list, int problem_count);

// registry.cuh:72-107: a (cfg string, function) list and a name -> function map
struct Kernel {
  std::string cfg_str;
  FuncType func;
  Kernel(std::string s, FuncType f) : cfg_str(std::move(s)), func(f) {}
};
struct KernelRegistry {
  std::vector<Kernel> storage_;
  std::unordered_map<std::string, FuncType> kernel_map_;
  size_t size() const { return storage_.size(); }
  const Kernel& operator[](size_t i) const { return storage_[i]; }
};
KernelRegistry& GetGlobalRegistry() {
  static KernelRegistry reg;
  return reg;
}
}  // namespace mxmoe

// ---- the translation unit a maintainer adds to the reference's `test` target ----
extern "C" int groupgemm_mxmoe(void**, void**, void**, void**, void**, void**, int64_t*, int64_t*, int64_t*,
                               int64_t*, dim3*, dim3*, mxmoe::QParams*, mxmoe::QParams*, int);
extern "C" const char* mxmoe_gg_last_error(void);

namespace {
void mxmoe_amd_gg(half** A, half** B, half** sa, half** sb, half** C, half** D, int64_t* la, int64_t* lb, int64_t* lc,
                  int64_t* ld, dim3* ps, dim3* hps, mxmoe::QParams* q, mxmoe::QParams* hq, int n) {
  if (groupgemm_mxmoe((void**)A, (void**)B, (void**)sa, (void**)sb, (void**)C, (void**)D, la, lb, lc, ld, ps, hps, q,
                      hq, n) != 0)
    throw std::runtime_error(mxmoe_gg_last_error());
}

struct RegisterMxmoeAmd {
  RegisterMxmoeAmd() {
    auto& reg = mxmoe::GetGlobalRegistry();
    const std::string name = "[mi355x: AUTO variant], groupgemm_mxmoe_amd";
    reg.storage_.emplace_back(name, &mxmoe_amd_gg);
    reg.kernel_map_[name] = &mxmoe_amd_gg;
  }
} register_mxmoe_amd;
}  // namespace
// ---- end of the INTEGRATION.md snippet ----

#define CHECK(x)                                                                                    \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) {                                                                         \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
      std::exit(3);                                                                                 \
    }                                                                                               \
  } while (0)

template <class T>
static T* dalloc(size_t n) {
  T* p = nullptr;
  CHECK(hipMalloc(&p, (n ? n : 1) * sizeof(T)));
  return p;
}
template <class T>
static T* upload(const std::vector<T>& v) {
  T* p = dalloc<T>(v.size());
  if (!v.empty()) CHECK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return p;
}

extern "C" int mxmoe_layout_check(void);  // layout_check.cpp

int main(int argc, char** argv) {
  if (argc == 2 && std::strcmp(argv[1], "--layout") == 0) {
    std::printf("{\"sizeof_QParams\": %zu, \"alignof_QParams\": %zu, \"offsetof_gsize\": %zu, \"offsetof_sym\": %zu, "
                "\"sizeof_dim3\": %zu, \"sizeof_half\": %zu, \"layout_check\": %d, \"registered\": %zu}\n",
                sizeof(mxmoe::QParams), alignof(mxmoe::QParams), offsetof(mxmoe::QParams, gsize),
                offsetof(mxmoe::QParams, sym), sizeof(dim3), sizeof(half), mxmoe_layout_check(),
                mxmoe::GetGlobalRegistry().size());
    return 0;
  }
  if (argc != 3) {
    std::fprintf(stderr, "usage: %s --layout | <in.bin> <out.bin>\n", argv[0]);
    return 2;
  }
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  auto rd = [&](void* p, size_t n) {
    if (n && std::fread(p, 1, n, f) != n) throw std::runtime_error("short read");
  };
  int32_t P = 0;
  rd(&P, 4);
  std::vector<dim3> h_problem_sizes(P);
  std::vector<mxmoe::QParams> qbits_list(P);
  for (int i = 0; i < P; ++i) {
    int32_t v[7];
    rd(v, sizeof v);
    h_problem_sizes[i] = dim3((unsigned)v[0], (unsigned)v[1], (unsigned)v[2]);
    qbits_list[i] = mxmoe::QParams(make_int2(v[3], v[4]), v[5], v[6] != 0);
    // the reference's QParams constructors leave the padding after `sym` uninitialised
    // (quantize.cuh:19-20): make it garbage on purpose, the library must not read it
    std::memset(reinterpret_cast<char*>(&qbits_list[i]) + offsetof(mxmoe::QParams, sym) + 1, 0xAB, 3);
  }
  // one buffer per operand with running offsets (test.cu:488-525): A / B in 16-bit words (the
  // reference's half* arithmetic on packed data), scale_zp = [sa(M) | sb(N)] per problem
  size_t words_a = 0, words_b = 0, elems_c = 0, elems_s = 0;
  std::vector<size_t> off_a(P), off_b(P), off_c(P), off_s(P), sz_a(P), sz_b(P), sz_sa(P), sz_sb(P);
  for (int i = 0; i < P; ++i) {
    const size_t M = h_problem_sizes[i].x, N = h_problem_sizes[i].y, K = h_problem_sizes[i].z;
    const int ab = qbits_list[i].qbits.x, wb = qbits_list[i].qbits.y;
    sz_a[i] = M * K * ab / 16;
    sz_b[i] = N * K * wb / 16;
    sz_sa[i] = ab >= 16 ? 0 : M;
    sz_sb[i] = wb >= 16 ? 0 : N;
    off_a[i] = words_a, off_b[i] = words_b, off_c[i] = elems_c, off_s[i] = elems_s;
    words_a += (sz_a[i] + 7) / 8 * 8;  // keep every problem's operands 16-B aligned
    words_b += (sz_b[i] + 7) / 8 * 8;
    elems_c += (M * N + 7) / 8 * 8;
    elems_s += (sz_sa[i] + sz_sb[i] + 7) / 8 * 8;
  }
  std::vector<uint16_t> hA(words_a), hB(words_b), hS(elems_s);
  for (int i = 0; i < P; ++i) {
    rd(hA.data() + off_a[i], sz_a[i] * 2);
    rd(hB.data() + off_b[i], sz_b[i] * 2);
    rd(hS.data() + off_s[i], sz_sa[i] * 2);
    rd(hS.data() + off_s[i] + sz_sa[i], sz_sb[i] * 2);
  }
  std::fclose(f);
  half* As = reinterpret_cast<half*>(upload(hA));
  half* Bs = reinterpret_cast<half*>(upload(hB));
  half* scale_zp = reinterpret_cast<half*>(upload(hS));
  half* Cs = dalloc<half>(elems_c);
  CHECK(hipMemset(Cs, 0xFF, (elems_c ? elems_c : 1) * sizeof(half)));  // NaN fill: every output must be written
  std::vector<half*> pA(P), pB(P), pSA(P), pSB(P), pC(P), pD(P);
  std::vector<int64_t> lda(P), ldb(P), ldc(P), ldd(P);
  for (int i = 0; i < P; ++i) {
    pA[i] = As + off_a[i];
    pB[i] = Bs + off_b[i];
    pSA[i] = scale_zp + off_s[i];
    pSB[i] = scale_zp + off_s[i] + sz_sa[i];
    pC[i] = pD[i] = Cs + off_c[i];
    lda[i] = h_problem_sizes[i].z, ldb[i] = h_problem_sizes[i].z, ldc[i] = ldd[i] = h_problem_sizes[i].y;
  }
  half** d_pA = upload(pA);
  half** d_pB = upload(pB);
  half** d_pSA = upload(pSA);
  half** d_pSB = upload(pSB);
  half** d_pC = upload(pC);
  half** d_pD = upload(pD);
  int64_t *d_lda = upload(lda), *d_ldb = upload(ldb), *d_ldc = upload(ldc), *d_ldd = upload(ldd);
  dim3* d_problem_sizes = upload(h_problem_sizes);
  mxmoe::QParams* d_qbits_list = upload(qbits_list);

  // test.cu:793-813: walk the registry, filter by name, call through the function pointer
  int ran = 0;
  const auto& reg = mxmoe::GetGlobalRegistry();
  for (size_t i = 0; i < reg.size(); ++i) {
    if (reg[i].cfg_str.find("mi355x") == std::string::npos) continue;
    std::printf("%s\n", reg[i].cfg_str.c_str());
    mxmoe::FuncType kernel = reg[i].func;
    try {
      kernel(d_pA, d_pB, d_pSA, d_pSB, d_pC, d_pD, d_lda, d_ldb, d_ldc, d_ldd, d_problem_sizes, h_problem_sizes.data(),
             d_qbits_list, qbits_list.data(), P);
    } catch (const std::exception& e) {
      std::fprintf(stderr, "kernel failed: %s\n", e.what());
      return 4;
    }
    ++ran;
  }
  CHECK(hipDeviceSynchronize());
  std::vector<uint16_t> hC(elems_c);
  if (elems_c) CHECK(hipMemcpy(hC.data(), Cs, elems_c * sizeof(half), hipMemcpyDeviceToHost));
  FILE* o = std::fopen(argv[2], "wb");
  if (!o) return 2;
  for (int i = 0; i < P; ++i) {
    const size_t n = (size_t)h_problem_sizes[i].x * h_problem_sizes[i].y;
    if (n && std::fwrite(hC.data() + off_c[i], 2, n, o) != n) return 2;
  }
  std::fclose(o);
  std::printf("{\"ran\": %d, \"problems\": %d}\n", ran, P);
  return ran == 1 ? 0 : 5;
}
