// ipc_probe.hip — probe of the primitives an IPC exchange between ranks needs (development tool):
// two processes (ranks 0/1, both on device `dev`) share buffers through hipIpc handles passed in
// files under `dir`; each iteration a kernel writes a block into the PEER's buffer, fences at
// system scope and bumps the peer's counter; the stream then waits on its own counter
// (hipStreamWaitValue32) and a kernel checks what the peer wrote.  Reports errors and us/iter,
// for coarse-grained and uncached allocations, eager and graph-captured waits.
//   hipcc --offload-arch=gfx950 -O3 tools/ipc_probe.hip -o tools/ipc_probe
//   ./tools/ipc_probe 0 /tmp/x & ./tools/ipc_probe 1 /tmp/x; wait
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <string>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "rank %d %s:%d %s: %s\n", g_rank, __FILE__, __LINE__, #x,         \
              hipGetErrorString(e_));                                                    \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)
static int g_rank = 0;

__global__ void k_push(float4* __restrict__ peer, int n4, float tag, uint32_t* peer_ctr,
                       uint32_t* done) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n4) peer[i] = make_float4(tag, (float)i, tag, (float)i);
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t prev = atomicAdd(done, 1u);
    if (prev == gridDim.x - 1) {  // last block: every block's writes are fenced
      *done = 0;
      __threadfence_system();
      __hip_atomic_fetch_add(peer_ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

__global__ void k_wait(const uint32_t* ctr, uint32_t target) {
  if (threadIdx.x == 0)
    while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < target)
      __builtin_amdgcn_s_sleep(1);
  __syncthreads();
}

__global__ void k_check(const float4* __restrict__ mine, int n4, float tag, int* err) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const float4 v = mine[i];
  if (v.x != tag || v.y != (float)i) atomicAdd(err, 1);
}

static void put_file(const std::string& p, const void* d, size_t n) {
  std::string tmp = p + ".tmp";
  FILE* f = fopen(tmp.c_str(), "wb");
  fwrite(d, 1, n, f);
  fclose(f);
  rename(tmp.c_str(), p.c_str());
}
static void get_file(const std::string& p, void* d, size_t n) {
  for (int k = 0; k < 6000; ++k) {
    FILE* f = fopen(p.c_str(), "rb");
    if (f) {
      const size_t r = fread(d, 1, n, f);
      fclose(f);
      if (r == n) return;
    }
    usleep(10000);
  }
  fprintf(stderr, "rank %d: timeout waiting for %s\n", g_rank, p.c_str());
  exit(2);
}

int main(int argc, char** argv) {
  g_rank = atoi(argv[1]);
  const std::string dir = argv[2];
  const int dev = argc > 3 ? atoi(argv[3]) : 0;
  const int peer = 1 - g_rank;
  CK(hipSetDevice(dev));
  int can_wait = 0;
  CK(hipDeviceGetAttribute(&can_wait, hipDeviceAttributeCanUseStreamWaitValue, dev));
  printf("rank %d: stream wait value supported: %d\n", g_rank, can_wait);
  const int n4 = 8 * 700 * 32;  // 8 peers x 700 rows x 512 B
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int variant = 0; variant < 3; ++variant) {
    const unsigned flags = variant == 0 ? hipDeviceMallocDefault : hipDeviceMallocUncached;
    const bool spin = variant == 2;
    float4* buf;
    uint32_t *ctr, *done;
    int* err;
    CK(hipExtMallocWithFlags((void**)&buf, sizeof(float4) * n4, flags));
    CK(hipExtMallocWithFlags((void**)&ctr, 256, hipDeviceMallocUncached));
    CK(hipMalloc(&done, 4));
    CK(hipMalloc(&err, 4));
    CK(hipMemset(ctr, 0, 256));
    CK(hipMemset(done, 0, 4));
    CK(hipMemset(err, 0, 4));
    CK(hipDeviceSynchronize());
    hipIpcMemHandle_t hb, hc;
    CK(hipIpcGetMemHandle(&hb, buf));
    CK(hipIpcGetMemHandle(&hc, ctr));
    const std::string me = dir + "/v" + std::to_string(variant) + "_r" + std::to_string(g_rank);
    const std::string pe = dir + "/v" + std::to_string(variant) + "_r" + std::to_string(peer);
    put_file(me + "_b", &hb, sizeof hb);
    put_file(me + "_c", &hc, sizeof hc);
    hipIpcMemHandle_t pb, pc;
    get_file(pe + "_b", &pb, sizeof pb);
    get_file(pe + "_c", &pc, sizeof pc);
    float4* pbuf;
    uint32_t* pctr;
    CK(hipIpcOpenMemHandle((void**)&pbuf, pb, hipIpcMemLazyEnablePeerAccess));
    CK(hipIpcOpenMemHandle((void**)&pctr, pc, hipIpcMemLazyEnablePeerAccess));
    const int iters = 2000;
    const unsigned blocks = (n4 + 255) / 256;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, s));
    for (int e = 0; e < iters; ++e) {
      const float tag = (float)(g_rank * 100000 + e + 1);
      const float ptag = (float)(peer * 100000 + e + 1);
      k_push<<<blocks, 256, 0, s>>>(pbuf, n4, tag, pctr, done);
      if (spin) k_wait<<<1, 64, 0, s>>>(ctr, (uint32_t)(e + 1));
      else CK(hipStreamWaitValue32(s, ctr, (uint32_t)(e + 1), hipStreamWaitValueGte, 0xFFFFFFFFu));
      k_check<<<blocks, 256, 0, s>>>(buf, n4, ptag, err);
      // the peer may overwrite buf only after this check: a second handshake
      k_push<<<1, 64, 0, s>>>(pbuf + 0, 0, 0.f, pctr + 32, done + 0);
      if (spin) k_wait<<<1, 64, 0, s>>>(ctr + 32, (uint32_t)(e + 1));
      else CK(hipStreamWaitValue32(s, ctr + 32, (uint32_t)(e + 1), hipStreamWaitValueGte, 0xFFFFFFFFu));
    }
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    int herr = 0;
    CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    printf("rank %d variant %s: %d iters, %.2f us/iter (2 pushes + 2 waits + check), errors %d\n",
           g_rank, variant == 0 ? "coarse" : variant == 1 ? "uncached" : "uncached+spin", iters, ms * 1e3 / iters, herr);
    // graph capture of a wait
    hipGraph_t gr = nullptr;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    const hipError_t ew = hipStreamWaitValue32(s, ctr, 0u, hipStreamWaitValueGte, 0xFFFFFFFFu);
    const hipError_t ee = hipStreamEndCapture(s, &gr);
    printf("rank %d: capture of hipStreamWaitValue32: wait=%s end=%s\n", g_rank, hipGetErrorString(ew),
           hipGetErrorString(ee));
    if (gr) {
      hipGraphExec_t ex = nullptr;
      const hipError_t ei = hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0);
      printf("rank %d: instantiate: %s\n", g_rank, hipGetErrorString(ei));
      if (ex) {
        CK(hipGraphLaunch(ex, s));
        CK(hipStreamSynchronize(s));
        (void)!hipGraphExecDestroy(ex);
      }
      (void)!hipGraphDestroy(gr);
    }
    (void)!hipGetLastError();
    CK(hipDeviceSynchronize());
    put_file(me + "_done", &herr, 4);
    int pdone;
    get_file(pe + "_done", &pdone, 4);
    CK(hipIpcCloseMemHandle(pbuf));
    CK(hipIpcCloseMemHandle(pctr));
  }
  return 0;
}
