// Which multi-stream capture patterns does this HIP runtime accept? (diagnostic for the
// engine's graph-capture path; one pattern per process: ./capture_patterns <k>)
//   1 fork to one side stream (event), kernel there, join back
//   2 fork to two side streams, a D2D memcpy on each, cross waits, join both
//   3 as 2, but one event recorded twice inside the capture (re-record after use)
//   4 an event recorded eagerly before the capture, re-recorded and waited inside it
//   5 a side stream that waits on the fork and gets no work (never joined)
//   6 as 2 with hipMemcpyAsync on a side stream that has only waited so far
//   7 the fork event itself re-recorded on the origin stream later in the capture
//   8 a side stream with work joined only indirectly (through another side stream)
//   9 the engine's P = 2 ring program as LocalWorld posts it: per rank a comm and a compute
//     stream, per tick pre / post / comm / reduce events, 1200-byte copies (argv[2] = ticks)
//  10 s1 records e1 after a kernel; s2 (with a node) waits e1; s1 captures nothing after e1
//  11 RingExecutor's direct shape, K = argv[2] slices: comm: group k (a kernel), record ce[k];
//     compute waits ce[k], fold k, record re[k]; then comm waits re[k] and allgather k — so comm
//     waits re[0] AFTER compute captured fold 1 .. K-1 behind it
//  12 s1 records e1 after a kernel, then captures another kernel; s2 (with a node) waits e1
//  13 as 12, but s2 has no node of its own when it waits e1
//  14 the minimal crash found by bisecting the engine's P = 3 program (tools/capture_replay.hip,
//     profiles/r03/graph/): three forked streams A B C record pA pB pC before any node; A waits
//     pC, copies, waits pB, copies; C copies, then waits pA; all joined. Every wait is on an event
//     recorded in the capture and every stream is joined — hipStreamEndCapture segfaults.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::printf("  %s -> %s\n", #x, hipGetErrorString(e_));                           \
            std::fflush(stdout);                                                               \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

__global__ void inc(float *p, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] += 1.0f;
}

int main(int argc, char **argv) {
    const int k = argc > 1 ? std::atoi(argv[1]) : 1;
    const int n = 1 << 16;
    float *a, *b, *c;
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&b, n * 4));
    CK(hipMalloc(&c, n * 4));
    CK(hipMemset(a, 0, n * 4));
    hipStream_t o, s1, s2;
    CK(hipStreamCreateWithFlags(&o, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t fork, e1, e2, j1, j2;
    for (hipEvent_t *e : {&fork, &e1, &e2, &j1, &j2}) CK(hipEventCreateWithFlags(e, hipEventDisableTiming));
    if (k == 4) {
        CK(hipEventRecord(e1, s1));
        CK(hipStreamSynchronize(s1));
    }
    std::printf("pattern %d: begin capture\n", k);
    std::fflush(stdout);
    CK(hipStreamBeginCapture(o, hipStreamCaptureModeGlobal));
    CK(hipEventRecord(fork, o));
    CK(hipStreamWaitEvent(s1, fork, 0));
    if (k != 1) CK(hipStreamWaitEvent(s2, fork, 0));
    switch (k) {
        case 1:
            hipLaunchKernelGGL(inc, dim3(n / 256), dim3(256), 0, s1, a, n);
            CK(hipEventRecord(j1, s1));
            CK(hipStreamWaitEvent(o, j1, 0));
            break;
        case 2:
        case 3:
        case 4:
        case 6:
        case 7:
            if (k != 6) hipLaunchKernelGGL(inc, dim3(n / 256), dim3(256), 0, s1, a, n);
            CK(hipEventRecord(e1, s1));
            if (k == 3) {
                CK(hipStreamWaitEvent(s2, e1, 0));
                hipLaunchKernelGGL(inc, dim3(n / 256), dim3(256), 0, s1, a, n);
                CK(hipEventRecord(e1, s1));  // re-recorded
            }
            CK(hipStreamWaitEvent(s2, e1, 0));
            CK(hipMemcpyAsync(b, a, n * 4, hipMemcpyDeviceToDevice, s2));
            CK(hipEventRecord(e2, s2));
            CK(hipStreamWaitEvent(s1, e2, 0));
            CK(hipMemcpyAsync(c, b, n * 4, hipMemcpyDeviceToDevice, s1));
            if (k == 7) {
                CK(hipEventRecord(fork, o));
                CK(hipStreamWaitEvent(s1, fork, 0));
            }
            CK(hipEventRecord(j1, s1));
            CK(hipEventRecord(j2, s2));
            CK(hipStreamWaitEvent(o, j1, 0));
            CK(hipStreamWaitEvent(o, j2, 0));
            break;
        case 8:
            hipLaunchKernelGGL(inc, dim3(n / 256), dim3(256), 0, s2, a, n);
            CK(hipEventRecord(e2, s2));
            CK(hipStreamWaitEvent(s1, e2, 0));
            CK(hipMemcpyAsync(c, a, n * 4, hipMemcpyDeviceToDevice, s1));
            CK(hipEventRecord(j1, s1));
            CK(hipStreamWaitEvent(o, j1, 0));  // s2 joined only through s1
            break;
        case 9: {
            const int T = argc > 2 ? std::atoi(argv[2]) : 2;
            hipStream_t cm[2], cp[2];
            hipEvent_t pre[2][4], post[2][4], cev[2][4], red[2][4], join[2];
            for (int r = 0; r < 2; ++r) {
                CK(hipStreamCreateWithFlags(&cm[r], hipStreamNonBlocking));
                CK(hipStreamCreateWithFlags(&cp[r], hipStreamNonBlocking));
                CK(hipEventCreateWithFlags(&join[r], hipEventDisableTiming));
                for (int t = 0; t < 4; ++t)
                    for (hipEvent_t *e : {&pre[r][t], &post[r][t], &cev[r][t], &red[r][t]})
                        CK(hipEventCreateWithFlags(e, hipEventDisableTiming));
            }
            float *buf[2] = {b, c};
            for (int r = 0; r < 2; ++r) {
                CK(hipStreamWaitEvent(cm[r], fork, 0));
                CK(hipStreamWaitEvent(cp[r], fork, 0));
            }
            for (int t = 0; t < T; ++t) {
                for (int r = 0; r < 2; ++r) {
                    if (t > 0) CK(hipStreamWaitEvent(cm[r], red[r][t - 1], 0));
                    CK(hipEventRecord(pre[r][t], cm[r]));
                }
                for (int r = 0; r < 2; ++r) {
                    CK(hipStreamWaitEvent(cm[r], pre[1 - r][t], 0));
                    CK(hipMemcpyAsync(buf[r] + 1024, buf[1 - r], 1200, hipMemcpyDeviceToDevice, cm[r]));
                    CK(hipEventRecord(post[r][t], cm[r]));
                }
                for (int r = 0; r < 2; ++r) CK(hipStreamWaitEvent(cm[r], post[1 - r][t], 0));
                for (int r = 0; r < 2; ++r) {
                    if (t == T - 1) break;
                    CK(hipEventRecord(cev[r][t], cm[r]));
                    CK(hipStreamWaitEvent(cp[r], cev[r][t], 0));
                    hipLaunchKernelGGL(inc, dim3(1), dim3(256), 0, cp[r], buf[r], 300);
                    CK(hipEventRecord(red[r][t], cp[r]));
                }
            }
            for (int r = 0; r < 2; ++r) {
                CK(hipEventRecord(join[r], cm[r]));
                CK(hipStreamWaitEvent(o, join[r], 0));
            }
            CK(hipMemcpyAsync(c, b, 4, hipMemcpyDeviceToDevice, o));
            break;
        }
        case 10:
        case 12:
        case 13:
            hipLaunchKernelGGL(inc, dim3(n / 256), dim3(256), 0, s1, a, n);
            CK(hipEventRecord(e1, s1));
            if (k != 10) hipLaunchKernelGGL(inc, dim3(n / 256), dim3(256), 0, s1, a, n);
            if (k != 13) hipLaunchKernelGGL(inc, dim3(n / 256), dim3(256), 0, s2, b, n);
            CK(hipStreamWaitEvent(s2, e1, 0));
            CK(hipMemcpyAsync(c, a, 4, hipMemcpyDeviceToDevice, s2));
            CK(hipEventRecord(j1, s1));
            CK(hipEventRecord(j2, s2));
            CK(hipStreamWaitEvent(o, j1, 0));
            CK(hipStreamWaitEvent(o, j2, 0));
            break;
        case 11: {  // s1 = comm, s2 = compute
            const int K = argc > 2 ? std::atoi(argv[2]) : 3;
            hipEvent_t ce[16], re[16];
            for (int i = 0; i < K; ++i) {
                CK(hipEventCreateWithFlags(&ce[i], hipEventDisableTiming));
                CK(hipEventCreateWithFlags(&re[i], hipEventDisableTiming));
            }
            for (int i = 0; i < K; ++i) {
                hipLaunchKernelGGL(inc, dim3(n / 256), dim3(256), 0, s1, a, n);  // RS group i
                CK(hipEventRecord(ce[i], s1));
                CK(hipStreamWaitEvent(s2, ce[i], 0));
                hipLaunchKernelGGL(inc, dim3(n / 256), dim3(256), 0, s2, b, n);  // fold i
                CK(hipEventRecord(re[i], s2));
            }
            for (int i = 0; i < K; ++i) {
                CK(hipStreamWaitEvent(s1, re[i], 0));
                hipLaunchKernelGGL(inc, dim3(n / 256), dim3(256), 0, s1, c, n);  // AG group i
            }
            CK(hipEventRecord(j1, s1));
            CK(hipEventRecord(j2, s2));
            CK(hipStreamWaitEvent(o, j1, 0));
            CK(hipStreamWaitEvent(o, j2, 0));
            break;
        }
        case 14: {
            hipStream_t s3;
            hipEvent_t pa, pb, pc, j3;
            CK(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));
            for (hipEvent_t *e : {&pa, &pb, &pc, &j3}) CK(hipEventCreateWithFlags(e, hipEventDisableTiming));
            CK(hipStreamWaitEvent(s3, fork, 0));  // A = s1, B = s2, C = s3 (s1, s2 waited above)
            CK(hipEventRecord(pa, s1));
            CK(hipEventRecord(pb, s2));
            CK(hipEventRecord(pc, s3));
            CK(hipStreamWaitEvent(s1, pc, 0));
            CK(hipMemcpyAsync(b, a, 256, hipMemcpyDeviceToDevice, s1));
            CK(hipStreamWaitEvent(s1, pb, 0));
            CK(hipMemcpyAsync(b + 64, a + 64, 256, hipMemcpyDeviceToDevice, s1));
            CK(hipMemcpyAsync(c, a, 432, hipMemcpyDeviceToDevice, s3));
            CK(hipStreamWaitEvent(s3, pa, 0));
            CK(hipEventRecord(j1, s1));
            CK(hipEventRecord(j2, s2));
            CK(hipEventRecord(j3, s3));
            CK(hipStreamWaitEvent(o, j1, 0));
            CK(hipStreamWaitEvent(o, j2, 0));
            CK(hipStreamWaitEvent(o, j3, 0));
            break;
        }
        case 5:
            hipLaunchKernelGGL(inc, dim3(n / 256), dim3(256), 0, s1, a, n);
            CK(hipEventRecord(j1, s1));
            CK(hipStreamWaitEvent(o, j1, 0));
            break;  // s2 waited on the fork and is never joined
    }
    hipGraph_t g = nullptr;
    std::printf("pattern %d: end capture\n", k);
    std::fflush(stdout);
    CK(hipStreamEndCapture(o, &g));
    hipGraphExec_t x;
    std::printf("pattern %d: instantiate\n", k);
    std::fflush(stdout);
    CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(x, o));
    CK(hipStreamSynchronize(o));
    float h = -1;
    CK(hipMemcpy(&h, c, 4, hipMemcpyDeviceToHost));
    std::printf("pattern %d: ok (c[0] = %g)\n", k, h);
    return 0;
}
