// Probe (GPU box): can RCCL point-to-point ops be captured into a hipGraph?
// world = 1 communicator, send/recv to self, eager then captured + replayed.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <cstdio>
#include <vector>
#define CK(x) do { auto e_ = (x); if (e_ != 0) { printf("FAIL %s -> %d\n", #x, (int)e_); return 1; } } while (0)
int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  printf("start\n");
  ncclUniqueId id;
  CK(ncclGetUniqueId(&id));
  ncclComm_t comm;
  printf("id ok\n");
  CK(ncclCommInitRank(&comm, 1, id, 0));
  printf("comm ok\n");
  const size_t n = 1 << 20;
  float *a, *b;
  CK(hipMalloc(&a, n * 4));
  CK(hipMalloc(&b, n * 4));
  std::vector<float> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = (float)i;
  CK(hipMemcpy(a, h.data(), n * 4, hipMemcpyHostToDevice));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  // eager
  CK(hipMemset(b, 0, n * 4));
  CK(ncclGroupStart());
  CK(ncclSend(a, n * 4, ncclInt8, 0, comm, s));
  CK(ncclRecv(b, n * 4, ncclInt8, 0, comm, s));
  CK(ncclGroupEnd());
  CK(hipStreamSynchronize(s));
  std::vector<float> r(n);
  CK(hipMemcpy(r.data(), b, n * 4, hipMemcpyDeviceToHost));
  printf("eager ok=%d\n", (int)(r[12345] == 12345.f && r[n - 1] == (float)(n - 1)));
  // captured
  CK(hipMemset(b, 0, n * 4));
  hipGraph_t g;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
  for (int rep = 0; rep < 3; ++rep) {
    CK(ncclGroupStart());
    CK(ncclSend(a, n * 4, ncclInt8, 0, comm, s));
    CK(ncclRecv(b, n * 4, ncclInt8, 0, comm, s));
    CK(ncclGroupEnd());
  }
  CK(hipStreamEndCapture(s, &g));
  hipGraphExec_t ge;
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int k = 0; k < 5; ++k) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  CK(hipMemcpy(r.data(), b, n * 4, hipMemcpyDeviceToHost));
  printf("graph ok=%d\n", (int)(r[12345] == 12345.f && r[n - 1] == (float)(n - 1)));
  // timing: eager vs graph per exchange of 1.5 MB
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const size_t m = 1572864;
  CK(hipEventRecord(e0, s));
  for (int k = 0; k < 100; ++k) {
    CK(ncclGroupStart()); CK(ncclSend(a, m, ncclInt8, 0, comm, s)); CK(ncclRecv(b, m, ncclInt8, 0, comm, s)); CK(ncclGroupEnd());
  }
  CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  printf("eager self-exchange 1.5 MB: %.2f us each\n", ms * 10.f);
  (void)hipGraphExecDestroy(ge);
  (void)hipGraphDestroy(g);
  printf("graph destroyed\n");
  CK(ncclCommDestroy(comm));
  printf("done\n");
  return 0;
}
