/*
 * oracle/ref_path_port.c — TEST / BASELINE INFRASTRUCTURE ONLY (bench.py's cpu leg).
 *
 * A C restatement ("port") of the reference's whole CPU allreduce path, timed under MPICH
 * loopback on the host cores, because the reference itself cannot be built here
 * (src/cpp/def.h:10 needs TensorFlow headers). Per step, every rank has the
 * same keyed fp32 requests registered; then, as the reference does:
 *   1. the 3-lap ring token (RingTokenCommunicateHandler.cc:133-318): READY(first key),
 *      SYNC(all keys, each rank intersects), COMMUNICATE — every hop is two MPI_Send /
 *      MPI_Recv pairs, a packed 10-byte {type, requestType, length} header then the key list
 *      (MPIRingTokenCommunication.cc:29-102); non-roots forward COMMUNICATE before running;
 *   2. the fusion plan (<= 2^31-1 bytes) and its execution (MPIRingTokenCommunication.cc:548-733):
 *      memcpy every tensor into the fusion buffer, MPI_Allreduce(MPI_SUM) in place of
 *      MPICommunicator::allreduce (MPICommunicator.cc:14-28), memcpy back out.
 * The reference runs the token on two background threads per communicator; this port runs
 * the same messages from the main thread, which leaves out the thread hand-offs (a lower bound
 * of the reference's cost).
 *
 * usage: mpiexec -n P ref_path_port <elements_per_tensor> <tensors> <reps>
 * prints (rank 0) one JSON line: {"P":..,"bytes":..,"best_ms":..,"mean_ms":..,"GiBs":..}
 */
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { TAG_META = 0, TAG_MSG = 1 };
enum { READY = 0, SYNC = 1, COMMUNICATE = 2 };

static void send_token(int to, unsigned char type, const char *msg, size_t len) {
    unsigned char meta[10];
    uint64_t l = len;
    meta[0] = type;
    meta[1] = 1; /* TOKEN_REQUEST_ALLREDUCE */
    memcpy(meta + 2, &l, 8);
    MPI_Send(meta, 10, MPI_BYTE, to, TAG_META, MPI_COMM_WORLD);
    MPI_Send(msg, (int)len, MPI_CHAR, to, TAG_MSG, MPI_COMM_WORLD);
}

static size_t recv_token(int from, unsigned char *type, char *buf, size_t cap) {
    unsigned char meta[10];
    uint64_t l;
    MPI_Recv(meta, 10, MPI_BYTE, from, TAG_META, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
    memcpy(&l, meta + 2, 8);
    if (l >= cap) { fprintf(stderr, "token too long\n"); MPI_Abort(MPI_COMM_WORLD, 2); }
    MPI_Recv(buf, (int)l, MPI_CHAR, from, TAG_MSG, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
    buf[l] = 0;
    *type = meta[0];
    return (size_t)l;
}

int main(int argc, char **argv) {
    int provided, rank, P, t, r, reps, ntens;
    size_t n, cap = 1 << 20, len;
    char *keys, *tok;
    float **in, **out, *fin, *fout;
    double best = 1e30, sum = 0;
    MPI_Init_thread(&argc, &argv, MPI_THREAD_MULTIPLE, &provided); /* MPIBackend.cc:77-86 */
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &P);
    if (argc != 4) { if (!rank) fprintf(stderr, "usage: %s elements tensors reps\n", argv[0]); MPI_Abort(MPI_COMM_WORLD, 1); }
    n = (size_t)strtoull(argv[1], NULL, 10);
    ntens = atoi(argv[2]);
    reps = atoi(argv[3]);
    in = malloc(sizeof(float *) * ntens);
    out = malloc(sizeof(float *) * ntens);
    for (t = 0; t < ntens; ++t) {
        size_t i;
        in[t] = malloc(n * 4);
        out[t] = malloc(n * 4);
        for (i = 0; i < n; ++i) in[t][i] = (float)(rank + 1) * 0.5f + (float)(i % 7);
    }
    fin = malloc(n * 4 * (size_t)ntens);
    fout = malloc(n * 4 * (size_t)ntens);
    memset(fin, 0, n * 4 * (size_t)ntens);
    memset(fout, 0, n * 4 * (size_t)ntens);
    keys = malloc(cap);
    tok = malloc(cap);
    len = 0;
    for (t = 0; t < ntens; ++t) len += (size_t)snprintf(keys + len, cap - len, "Allreduce::grad_%05d\n", t);
    for (r = -1; r < reps; ++r) { /* r = -1: warm-up */
        int succ = (rank + 1) % P, pred = (rank + P - 1) % P;
        unsigned char type;
        double t0;
        MPI_Barrier(MPI_COMM_WORLD);
        t0 = MPI_Wtime();
        if (P > 1) {
            if (rank == 0) {
                send_token(succ, READY, "grad_00000", 10);
                recv_token(pred, &type, tok, cap);
                send_token(succ, SYNC, keys, len);
                recv_token(pred, &type, tok, cap);
                send_token(succ, COMMUNICATE, tok, strlen(tok));
            } else {
                size_t l = recv_token(pred, &type, tok, cap);   /* READY: key registered here */
                send_token(succ, type, tok, l);
                l = recv_token(pred, &type, tok, cap);          /* SYNC: intersection (all present) */
                send_token(succ, type, tok, l);
                l = recv_token(pred, &type, tok, cap);          /* COMMUNICATE: forward first */
                send_token(succ, type, tok, l);
            }
        }
        /* executeCommunicatePlan_: one plan (total < 2^31-1 bytes), memcpy in / allreduce / out */
        for (t = 0; t < ntens; ++t) memcpy(fin + (size_t)t * n, in[t], n * 4);
        MPI_Allreduce(fin, fout, (int)(n * (size_t)ntens), MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD);
        for (t = 0; t < ntens; ++t) memcpy(out[t], fout + (size_t)t * n, n * 4);
        if (P > 1 && rank == 0) recv_token(pred, &type, tok, cap); /* COMMUNICATE returns */
        {
            double dt = MPI_Wtime() - t0, mx;
            MPI_Allreduce(&dt, &mx, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
            if (r >= 0) {
                sum += mx;
                if (mx < best) best = mx;
            }
        }
    }
    if (rank == 0) {
        double bytes = (double)n * 4.0 * ntens;
        double expect0 = 0.5 * (double)P * (P + 1) / 2.0; /* element 0: sum of 0.5*(r+1) */
        printf("{\"P\": %d, \"bytes\": %.0f, \"tensors\": %d, \"best_ms\": %.4f, \"mean_ms\": %.4f, "
               "\"GiBs\": %.4f, \"check_out0\": %.3f, \"expect_out0\": %.3f}\n",
               P, bytes, ntens, best * 1e3, sum / reps * 1e3, bytes / best / 1073741824.0, out[0][0], expect0);
    }
    MPI_Finalize();
    return 0;
}
