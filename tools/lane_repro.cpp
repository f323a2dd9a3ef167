// Isolated replay of the executor's side-lane capture (csrc/exec.hip run_ops / edgedet_graph_create)
// to find which destruction made a later hipGraphLaunch segfault in round 3:
// capture on a caller stream that forks two side streams with an event, runs a kernel on each side
// stream and on the caller stream, joins them back with one event per side stream (the FORK / JOIN
// records), instantiates and uploads the graph; then destroys the side STREAMS, or the fork / join
// EVENTS, or both, or nothing; then launches the graph three times and checks the kernels' output.
// Plain HIP runtime, no library, one variant per process:
//
//   lane_repro none|events|streams|both                 (destroyed after instantiate + upload)
//   lane_repro streams_during|events_during             (destroyed after the JOIN, BEFORE
//                                                         hipStreamEndCapture: the round-3 library
//                                                         released a run's lane set when run_ops
//                                                         returned, inside the capture)
//
// Exit 0 = the graph ran and the results are right after the destruction; 2 = wrong results; 3 = a
// HIP error.  A segfault shows as the process dying (status 139 from the shell).
//
// Build: hipcc -O2 --offload-arch=gfx950 tools/lane_repro.cpp -o tools/lane_repro
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#define CK(e)                                                                                   \
    do {                                                                                        \
        hipError_t r_ = (e);                                                                    \
        if (r_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #e, hipGetErrorString(r_)); \
            return 3;                                                                           \
        }                                                                                       \
    } while (0)

__global__ void fill(float* y, int n, float v) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = y[i] * 0.5f + v;  // depends on the previous value: a lost or repeated node shows
}

int main(int argc, char** argv) {
    const char* mode = argc > 1 ? argv[1] : "none";
    const bool kill_streams = !strcmp(mode, "streams") || !strcmp(mode, "both");
    const bool kill_events = !strcmp(mode, "events") || !strcmp(mode, "both");
    const bool during_streams = !strcmp(mode, "streams_during"), during_events = !strcmp(mode, "events_during");
    constexpr int N = 1 << 16, SIDE = 2;
    float* buf = nullptr;
    CK(hipMalloc(&buf, sizeof(float) * N * (SIDE + 1)));
    CK(hipMemset(buf, 0, sizeof(float) * N * (SIDE + 1)));
    hipStream_t s, side[SIDE];
    hipEvent_t fork_ev, join_ev[SIDE];
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int l = 0; l < SIDE; ++l) {
        CK(hipStreamCreateWithFlags(&side[l], hipStreamNonBlocking));
        CK(hipEventCreateWithFlags(&join_ev[l], hipEventDisableTiming));
    }
    CK(hipEventCreateWithFlags(&fork_ev, hipEventDisableTiming));

    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    CK(hipEventRecord(fork_ev, s));  // FORK
    for (int l = 0; l < SIDE; ++l) CK(hipStreamWaitEvent(side[l], fork_ev, 0));
    for (int l = 0; l < SIDE; ++l)
        hipLaunchKernelGGL(fill, dim3(N / 256), dim3(256), 0, side[l], buf + (l + 1) * N, N, (float)(l + 1));
    hipLaunchKernelGGL(fill, dim3(N / 256), dim3(256), 0, s, buf, N, 10.f);
    for (int l = 0; l < SIDE; ++l) {  // JOIN
        CK(hipEventRecord(join_ev[l], side[l]));
        CK(hipStreamWaitEvent(s, join_ev[l], 0));
    }
    if (during_streams)
        for (int l = 0; l < SIDE; ++l) CK(hipStreamDestroy(side[l]));
    if (during_events) {
        CK(hipEventDestroy(fork_ev));
        for (int l = 0; l < SIDE; ++l) CK(hipEventDestroy(join_ev[l]));
    }
    CK(hipStreamEndCapture(s, &graph));
    CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    CK(hipGraphUpload(exec, s));
    CK(hipStreamSynchronize(s));
    printf("captured; destroying %s\n", mode);
    fflush(stdout);
    if (kill_streams)
        for (int l = 0; l < SIDE; ++l) CK(hipStreamDestroy(side[l]));
    if (kill_events) {
        CK(hipEventDestroy(fork_ev));
        for (int l = 0; l < SIDE; ++l) CK(hipEventDestroy(join_ev[l]));
    }
    for (int r = 0; r < 3; ++r) {
        CK(hipGraphLaunch(exec, s));
        printf("launch %d issued\n", r);
        fflush(stdout);
    }
    CK(hipStreamSynchronize(s));
    std::vector<float> h((size_t)N * (SIDE + 1));
    CK(hipMemcpy(h.data(), buf, sizeof(float) * h.size(), hipMemcpyDeviceToHost));
    // three applications of y = y / 2 + v from 0: v * (1 + 1/2 + 1/4) = 1.75 v
    int bad = 0;
    for (int l = 0; l <= SIDE; ++l) {
        const float want = 1.75f * (l == 0 ? 10.f : (float)l);
        for (int i = 0; i < N; ++i) bad += h[(size_t)l * N + i] != want;
    }
    printf("mode %s: %s (%d wrong values)\n", mode, bad ? "WRONG" : "ok", bad);
    CK(hipGraphExecDestroy(exec));
    CK(hipGraphDestroy(graph));
    CK(hipFree(buf));
    return bad ? 2 : 0;
}
