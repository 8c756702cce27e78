// Pure-HIP probe for the round-4 hipGraphLaunch segfault (gpurun_out/r4m):
// several live "models", each owning two auxiliary streams and a pool of events, capture a
// ~90-node graph whose kernels fork over three lanes (the capture stream + the two aux streams,
// joined back by events, exactly the pattern of run_dag in csrc/detector.hip), instantiate it and
// launch it on a launch stream.  Mode "destroy" destroys the capture stream right after
// hipStreamEndCapture (the round-4 code); mode "keep" keeps one capture stream per model alive
// for the model's lifetime (the round-5 code).
//
// build: hipcc -O2 --offload-arch=gfx950 tools/graph_fork_repro.hip -o tools/_graph_fork_repro
// run:   tools/_graph_fork_repro destroy|keep [models=8] [launches=4]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                       \
    }                                                                                \
  } while (0)

__global__ void bump(int* p, int i) {
  if (threadIdx.x == 0) p[i] += 1;
}

struct Model {
  std::vector<hipStream_t> aux;
  std::vector<hipEvent_t> ev;
  hipStream_t cap = nullptr;  // "keep" mode
  std::vector<hipGraphExec_t> execs;
  int* buf = nullptr;
};

constexpr int NT = 90, LANES = 3;

static void record(Model& m, hipStream_t st) {
  hipEvent_t fork = m.ev[NT];
  CK(hipEventRecord(fork, st));
  for (int l = 1; l < LANES; ++l) CK(hipStreamWaitEvent(m.aux[l - 1], fork, 0));
  auto lane_stream = [&](int l) { return l == 0 ? st : m.aux[l - 1]; };
  for (int t = 0; t < NT; ++t) {
    const int lane = (t / 3) % LANES;
    hipStream_t s = lane_stream(lane);
    if (t > 0 && ((t - 1) / 3) % LANES != lane) CK(hipStreamWaitEvent(s, m.ev[t - 1], 0));
    hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, s, m.buf, t);
    CK(hipGetLastError());
    CK(hipEventRecord(m.ev[t], s));
  }
  for (int l = 1; l < LANES; ++l) {
    CK(hipEventRecord(m.ev[NT + l], m.aux[l - 1]));
    CK(hipStreamWaitEvent(st, m.ev[NT + l], 0));
  }
}

static hipGraphExec_t capture(Model& m, bool keep) {
  hipStream_t cap;
  if (keep) {
    if (!m.cap) CK(hipStreamCreateWithFlags(&m.cap, hipStreamNonBlocking));
    cap = m.cap;
  } else {
    CK(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
  }
  hipGraph_t g;
  CK(hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal));
  record(m, cap);
  CK(hipStreamEndCapture(cap, &g));
  if (!keep) CK(hipStreamDestroy(cap));
  hipGraphExec_t ge;
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphDestroy(g));
  return ge;
}

int main(int argc, char** argv) {
  const bool keep = argc > 1 && !strcmp(argv[1], "keep");
  const int n_models = argc > 2 ? atoi(argv[2]) : 8;
  const int launches = argc > 3 ? atoi(argv[3]) : 4;
  std::vector<Model> models(n_models);
  std::vector<hipStream_t> launch(4);
  for (auto& s : launch) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int total = 0;
  for (int i = 0; i < n_models; ++i) {
    Model& m = models[i];
    m.aux.resize(LANES - 1);
    for (auto& s : m.aux) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    m.ev.resize(NT + LANES + 1);
    for (auto& e : m.ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CK(hipMalloc(&m.buf, NT * sizeof(int)));
    CK(hipMemset(m.buf, 0, NT * sizeof(int)));
    for (int k = 0; k < 2; ++k) m.execs.push_back(capture(m, keep));  // two graphs per model
    // launch every live model's graphs on the launch streams, several at a time in flight
    for (int r = 0; r < launches; ++r)
      for (int j = 0; j <= i; ++j)
        for (size_t k = 0; k < models[j].execs.size(); ++k) {
          CK(hipGraphLaunch(models[j].execs[k], launch[(j + k) % launch.size()]));
          ++total;
        }
    CK(hipDeviceSynchronize());
    printf("model %d: %d graph launches so far\n", i + 1, total);
    fflush(stdout);
  }
  // every bump ran exactly once per launch of a graph of that model
  int bad = 0;
  for (int i = 0; i < n_models; ++i) {
    std::vector<int> h(NT);
    CK(hipMemcpy(h.data(), models[i].buf, NT * sizeof(int), hipMemcpyDeviceToHost));
    const int want = 2 * launches * (n_models - i);
    for (int t = 0; t < NT; ++t) bad += h[t] != want;
  }
  printf("%s: %d models, %d launches, %d wrong counters\n", keep ? "keep" : "destroy", n_models, total, bad);
  return bad ? 1 : 0;
}
