// Diagnostic: time parse_candidate (pqg_scan.hip, K1a') per header candidate
// of one column chunk on the GPU, one lane per candidate, and print the
// slowest.  Build: hipcc -O3 --offload-arch=gfx950 -I../include -I../parquet-go_amd/csrc
//   cand_timing.hip -o cand_timing;  run: ./cand_timing <chunk.bin> [tcs [all.txt [per_lane]]]
#include "pqg_scan.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

namespace pqg {
__global__ void __launch_bounds__(256) k_cand_time(JobDev* job, const int64_t* pos, int n, Cand* out,
                                                   uint64_t* cycles, int per_lane) {
  __shared__ SkipFrame frames[256][kCandFrames];
  __shared__ int16_t lasts[256][kCandLast];
  __shared__ __attribute__((aligned(16))) uint8_t wins[256][16 * kCandWin];
  // per_lane: one candidate per lane, as k_cand_parse (the wave's clock is
  // its slowest lane's); else one per wave (lane 0: the candidate's own clock)
  const int i = per_lane ? blockIdx.x * 256 + threadIdx.x : blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n || (!per_lane && (threadIdx.x & 63))) return;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  parse_candidate(*job, pos[i], frames[threadIdx.x], lasts[threadIdx.x], lds_ptr(wins[threadIdx.x]), &out[i]);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  cycles[i] = t1 - t0;
}
}  // namespace pqg

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 1;
  std::vector<uint8_t> b;
  int c;
  while ((c = fgetc(f)) != EOF) b.push_back((uint8_t)c);
  fclose(f);
  const int64_t n = (int64_t)b.size();
  std::vector<int64_t> pos;
  for (int64_t p = 0; p + 2 < n; p++)
    if (b[p] == 0x15 && (b[p + 1] & 0xf9) == 0 && b[p + 2] == 0x15) pos.push_back(p);
  printf("%zu candidates in %ld bytes\n", pos.size(), (long)n);
  uint8_t* d;
  CK(hipMalloc(&d, n + 64));
  CK(hipMemcpy(d, b.data(), n, hipMemcpyHostToDevice));
  pqg::JobDev job{};
  job.data = d;
  job.data_len = n;
  job.tcs = argc > 2 && atoll(argv[2]) > 0 ? atoll(argv[2]) : n;
  job.type = 1;  // INT32
  job.type_length = 0;
  job.max_def = 1;
  job.codec = 0;
  job.value_width = 4;
  pqg::JobDev* dj;
  CK(hipMalloc(&dj, sizeof(job)));
  CK(hipMemcpy(dj, &job, sizeof(job), hipMemcpyHostToDevice));
  int64_t* dp;
  pqg::Cand* dc;
  uint64_t* dcy;
  const int m = (int)pos.size();
  CK(hipMalloc(&dp, 8 * (size_t)m + 8));
  CK(hipMalloc(&dc, sizeof(pqg::Cand) * (size_t)m + 8));
  CK(hipMalloc(&dcy, 8 * (size_t)m + 8));
  CK(hipMemcpy(dp, pos.data(), 8 * (size_t)m, hipMemcpyHostToDevice));
  const int per_lane = argc > 4 && atoi(argv[4]) != 0;
  for (int rep = 0; rep < 2; rep++) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(pqg::k_cand_time, dim3(per_lane ? (m + 255) / 256 : (m + 3) / 4), dim3(256), 0, 0, dj, dp, m, dc,
                       dcy, per_lane);
    CK(hipEventRecord(e1, 0));
    CK(hipDeviceSynchronize());
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("rep %d: %.3f ms\n", rep, ms);
  }
  std::vector<uint64_t> cy(m);
  std::vector<pqg::Cand> cs(m);
  CK(hipMemcpy(cy.data(), dcy, 8 * (size_t)m, hipMemcpyDeviceToHost));
  CK(hipMemcpy(cs.data(), dc, sizeof(pqg::Cand) * (size_t)m, hipMemcpyDeviceToHost));
  std::vector<int> ord(m);
  for (int i = 0; i < m; i++) ord[i] = i;
  std::sort(ord.begin(), ord.end(), [&](int a, int b2) { return cy[a] > cy[b2]; });
  for (int k = 0; k < std::min(m, 12); k++) {
    const int i = ord[k];
    printf("pos %ld cycles %lu status %d type %d next %ld payload %ld bytes:", (long)pos[i], (unsigned long)cy[i],
           cs[i].status, cs[i].type, (long)cs[i].next, (long)cs[i].payload);
    for (int j = 0; j < 24 && pos[i] + j < n; j++) printf(" %02x", b[pos[i] + j]);
    printf("\n");
  }
  if (argc > 3) {  // every candidate: pos status type csize num_values payload next cycles
    FILE* o = fopen(argv[3], "w");
    for (int i = 0; i < m; i++)
      fprintf(o, "%ld %d %d %d %d %ld %ld %lu\n", (long)pos[i], cs[i].status, cs[i].type, cs[i].csize, cs[i].num_values,
              (long)cs[i].payload, (long)cs[i].next, (unsigned long)cy[i]);
    fclose(o);
  }
  return 0;
}
