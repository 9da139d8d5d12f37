// tune_zero_copy.hip — can the FEC kernels read their packets straight from
// pinned host memory (zero-copy over PCIe) as fast as a staged H2D copy moves
// them?  Measures, on 2^16 groups x 10 x 1350 B (885 MB) in pinned host memory:
//   * hipMemcpyAsync H2D / D2H of the rows (the staged path's transfer)
//   * stream_probe read of the host rows from a kernel (coherent and
//     non-coherent pinned memory)
//   * fixed encode with rows on the host, parity to device / to host
//   * ragged encode (configs[3] shapes) with packet bytes on the host
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/tune_zero_copy.hip -o tools/tune/build/tune_zero_copy
#include "../../libquic_amd/csrc/qfec_kernels.hip"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                            \
    }                                                                                          \
  } while (0)

template <typename F>
static double time_ms(F f, int reps) {
  f();
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const uint64_t G = argc > 1 ? atoll(argv[1]) : (1 << 16);
  const uint32_t k = 10, L = 1350;
  const uint64_t nb = G * k * L;
  const int reps = 5;
  uint8_t *h_coh, *h_nc, *d_rows, *d_par, *h_par;
  uint32_t* d_err;
  CK(hipHostMalloc(&h_coh, nb, hipHostMallocDefault));
  CK(hipHostMalloc(&h_nc, nb, hipHostMallocNonCoherent));
  CK(hipMalloc(&d_rows, nb));
  CK(hipMalloc(&d_par, G * 1452));
  CK(hipHostMalloc(&h_par, G * 1452, hipHostMallocDefault));
  CK(hipMalloc(&d_err, 4));
  CK(hipMemset(d_err, 0, 4));
  CK(qfec::launch_synth_fixed(d_rows, k, L, L, (uint64_t)k * L, 0, G, 0x51554943, 0));
  CK(hipMemcpy(h_coh, d_rows, nb, hipMemcpyDeviceToHost));
  CK(hipMemcpy(h_nc, d_rows, nb, hipMemcpyDeviceToHost));
  auto gbs = [&](double bytes, double ms) { return bytes / ms / 1e6; };
  std::printf("G %llu groups, %.0f MB rows\n", (unsigned long long)G, nb / 1e6);
  double ms = time_ms([&] { CK(hipMemcpyAsync(d_rows, h_coh, nb, hipMemcpyHostToDevice, 0)); }, reps);
  std::printf("%-44s %8.3f ms %8.1f GB/s\n", "H2D memcpy (coherent pinned)", ms, gbs(nb, ms));
  ms = time_ms([&] { CK(hipMemcpyAsync(h_coh, d_rows, nb, hipMemcpyDeviceToHost, 0)); }, reps);
  std::printf("%-44s %8.3f ms %8.1f GB/s\n", "D2H memcpy (coherent pinned)", ms, gbs(nb, ms));
  {  // both directions at once (two streams): the fused FEC + AEAD leg's budget
    uint8_t* h2;
    uint8_t* d2;
    CK(hipHostMalloc(&h2, nb, hipHostMallocDefault));
    CK(hipMalloc(&d2, nb));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    auto both = [&] {
      CK(hipMemcpyAsync(d_rows, h_coh, nb, hipMemcpyHostToDevice, s1));
      CK(hipMemcpyAsync(h2, d2, nb, hipMemcpyDeviceToHost, s2));
      CK(hipStreamSynchronize(s1));
      CK(hipStreamSynchronize(s2));
    };
    both();
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < reps; ++i) both();
    const double ms2 =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() /
        reps;
    std::printf("%-44s %8.3f ms %8.1f GB/s (each way %.1f)\n", "H2D || D2H (two streams)", ms2,
                gbs(2.0 * nb, ms2), gbs(nb, ms2));
    CK(hipHostFree(h2));
    CK(hipFree(d2));
  }
  for (int nc = 0; nc < 2; ++nc) {
    uint8_t* h = nc ? h_nc : h_coh;
    const char* tag = nc ? "non-coherent" : "coherent";
    char name[128];
    ms = time_ms([&] { CK(qfec::launch_stream_probe(h, nb, d_par, false, 0)); }, reps);
    std::snprintf(name, sizeof name, "kernel read of host rows (%s)", tag);
    std::printf("%-44s %8.3f ms %8.1f GB/s\n", name, ms, gbs(nb, ms));
    qfec::FixedArgs a{};
    a.rows = h;
    a.out = d_par;
    a.row_stride = L;
    a.group_stride = (uint64_t)k * L;
    a.parity_stride = L;
    a.out_stride = L;
    a.n_groups = G;
    a.k = k;
    a.L = L;
    a.err = d_err;
    ms = time_ms([&] { CK(qfec::launch_fixed(a, true, 0)); }, reps);
    std::snprintf(name, sizeof name, "fixed encode, rows on host (%s)", tag);
    std::printf("%-44s %8.3f ms %8.1f GB/s\n", name, ms, gbs(G * (k * L + L), ms));
    a.out = h_par;
    ms = time_ms([&] { CK(qfec::launch_fixed(a, true, 0)); }, reps);
    std::snprintf(name, sizeof name, "fixed encode, rows+parity on host (%s)", tag);
    std::printf("%-44s %8.3f ms %8.1f GB/s\n", name, ms, gbs(G * (k * L + L), ms));
    a.out = d_par;
    ms = time_ms([&] { CK(qfec::launch_fixed(a, false, 0)); }, reps);
    std::snprintf(name, sizeof name, "fixed encode cached, rows on host (%s)", tag);
    std::printf("%-44s %8.3f ms %8.1f GB/s\n", name, ms, gbs(G * (k * L + L), ms));
  }
  // ragged: CSR over the host rows (10 packets of 1350 per group = the fixed
  // bytes), tables on the device
  std::vector<uint64_t> off(G * k), poff(G);
  std::vector<uint16_t> len(G * k, (uint16_t)L);
  std::vector<uint32_t> ptr(G + 1);
  for (uint64_t g = 0; g <= G; ++g) ptr[g] = (uint32_t)(g * k);
  for (uint64_t p = 0; p < G * k; ++p) off[p] = p * L;
  for (uint64_t g = 0; g < G; ++g) poff[g] = g * 1452;
  uint64_t *d_off, *d_poff;
  uint16_t *d_len, *d_plen;
  uint32_t* d_ptr;
  CK(hipMalloc(&d_off, off.size() * 8));
  CK(hipMalloc(&d_poff, poff.size() * 8));
  CK(hipMalloc(&d_len, len.size() * 2));
  CK(hipMalloc(&d_plen, G * 2));
  CK(hipMalloc(&d_ptr, ptr.size() * 4));
  CK(hipMemcpy(d_off, off.data(), off.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_poff, poff.data(), poff.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_len, len.data(), len.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_ptr, ptr.data(), ptr.size() * 4, hipMemcpyHostToDevice));
  for (int where = 0; where < 3; ++where) {
    qfec::RaggedArgs r{};
    r.bytes = where == 0 ? d_rows : where == 1 ? h_coh : h_nc;
    r.pkt_off = d_off;
    r.pkt_len = d_len;
    r.grp_ptr = d_ptr;
    r.parity_off = d_poff;
    r.parity_len_out = d_plen;
    r.out = d_par;
    r.n_groups = G;
    r.err = d_err;
    ms = time_ms([&] { CK(qfec::launch_ragged(r, false, 0)); }, reps);
    const char* nm[] = {"ragged encode, bytes on device", "ragged encode, bytes on host (coherent)",
                        "ragged encode, bytes on host (non-coherent)"};
    std::printf("%-44s %8.3f ms %8.1f GB/s\n", nm[where], ms, gbs(G * (k * L + L), ms));
  }
  // correctness of one host-read encode vs the device-read one
  std::vector<uint8_t> p1(G * 1452), p2(G * 1452);
  qfec::FixedArgs a{};
  a.rows = d_rows; a.out = d_par; a.row_stride = L; a.group_stride = (uint64_t)k * L;
  a.parity_stride = L; a.out_stride = L; a.n_groups = G; a.k = k; a.L = L; a.err = d_err;
  CK(qfec::launch_fixed(a, true, 0));
  CK(hipMemcpy(p1.data(), d_par, G * L, hipMemcpyDeviceToHost));
  a.rows = h_coh; a.out = h_par;
  CK(qfec::launch_fixed(a, true, 0));
  CK(hipDeviceSynchronize());
  std::printf("host-read parity == device-read parity: %s\n",
              std::memcmp(p1.data(), h_par, G * L) == 0 ? "yes" : "NO");
  return 0;
}
