// What HIP records when a stream capture holds a hipMemsetAsync ahead of kernels on the same stream
// (round 3's first UpdateIO pipeline form: profiles/r04_graph_probe.txt).  Captures two forms, dumps
// each graph's nodes (types), roots and edges, and never instantiates or launches either:
//   A: hipMemsetAsync(scan words) -> kernel -> kernel      (the round-3 form that faulted on replay)
//   B: zero kernel -> kernel -> kernel                      (the form the engine captures now)
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/graph_probe scripts/graph_probe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

__global__ void zero_k(uint32_t *p, uint32_t n) {
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) p[i] = 0;
}
__global__ void step_k(uint32_t *p) {
  if (threadIdx.x == 0) atomicAdd(p, 1u);
}

static const char *type_name(hipGraphNodeType t) {
  switch (t) {
    case hipGraphNodeTypeKernel: return "kernel";
    case hipGraphNodeTypeMemcpy: return "memcpy";
    case hipGraphNodeTypeMemset: return "memset";
    case hipGraphNodeTypeEmpty: return "empty";
    default: return "other";
  }
}

static int dump(const char *name, hipGraph_t g) {
  size_t nn = 0, nr = 0, ne = 0;
  if (hipGraphGetNodes(g, nullptr, &nn) || hipGraphGetRootNodes(g, nullptr, &nr) ||
      hipGraphGetEdges(g, nullptr, nullptr, &ne))
    return 1;
  std::vector<hipGraphNode_t> nodes(nn), roots(nr), from(ne), to(ne);
  if ((nn && hipGraphGetNodes(g, nodes.data(), &nn)) || (nr && hipGraphGetRootNodes(g, roots.data(), &nr)) ||
      (ne && hipGraphGetEdges(g, from.data(), to.data(), &ne)))
    return 1;
  auto idx = [&](hipGraphNode_t x) {
    for (size_t i = 0; i < nn; ++i)
      if (nodes[i] == x) return (int)i;
    return -1;
  };
  printf("%s: %zu nodes, %zu roots, %zu edges\n", name, nn, nr, ne);
  for (size_t i = 0; i < nn; ++i) {
    hipGraphNodeType t;
    if (hipGraphNodeGetType(nodes[i], &t)) return 1;
    printf("  node %zu: %s\n", i, type_name(t));
  }
  for (size_t i = 0; i < nr; ++i) printf("  root: node %d\n", idx(roots[i]));
  for (size_t e = 0; e < ne; ++e) printf("  edge: node %d -> node %d\n", idx(from[e]), idx(to[e]));
  return 0;
}

int main() {
  uint32_t *d;
  if (hipMalloc(&d, 4096) != hipSuccess) return 1;
  hipStream_t st;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 1;
  for (int form = 0; form < 2; ++form) {
    if (hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed) != hipSuccess) return 1;
    if (form == 0) {
      if (hipMemsetAsync(d, 0, 256, st) != hipSuccess) return 1;
    } else {
      hipLaunchKernelGGL(zero_k, dim3(1), dim3(256), 0, st, d, 64u);
    }
    hipLaunchKernelGGL(step_k, dim3(4), dim3(64), 0, st, d);
    hipLaunchKernelGGL(step_k, dim3(4), dim3(64), 0, st, d + 1);
    hipGraph_t g = nullptr;
    if (hipStreamEndCapture(st, &g) != hipSuccess || !g) return 1;
    if (dump(form == 0 ? "A (hipMemsetAsync head)" : "B (zero kernel head)", g)) return 1;
    (void)hipGraphDestroy(g);  // never instantiated, never launched
  }
  return 0;
}
