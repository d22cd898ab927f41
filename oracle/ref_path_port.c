/*
 * oracle/ref_path_port.c — TEST / BASELINE INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).
 *
 * A C restatement ("port") of the reference's whole CPU allreduce path, timed under MPICH
 * loopback on the host cores, because the reference itself cannot be built here
 * (src/cpp/def.h:10 needs TensorFlow headers). It keeps the reference's
 * structure, so its cost includes what the reference pays besides MPI:
 *   * per communicator a handler with two threads (RingTokenCommunicateHandler.cc:13-32): a
 *     send thread that sleeps on a condition variable over the outgoing token queue and sends
 *     every queued token to rank+1 (sendMain_, :50-104), and a recv thread that receives tokens
 *     from rank-1 and runs the token state machine (recvMain_, :106-131), on a duplicate of
 *     MPI_COMM_WORLD (MPIBackend.cc wraps a copy of the world communicator);
 *   * the 3-lap ring token: rank 0 sends READY(first registered key) when a request arrives in
 *     WAITING_TENSORS (handleRequest, :327-363); a non-root forwards READY once that key is
 *     registered, else parks it until handleRequest sees it (:225-250); rank 0 answers READY
 *     with SYNC(all its registered keys) (:137-163); each non-root intersects and forwards
 *     (:251-300); rank 0 turns SYNC into COMMUNICATE (:165-181); non-roots forward
 *     COMMUNICATE, then communicate (:302-310); rank 0 communicates when COMMUNICATE returns,
 *     then READYs its next registered key or waits (:182-211);
 *   * every hop is two MPI_Send / MPI_Recv: a packed 10-byte {type, requestType, length}
 *     header then the "Allreduce::<key>\n" list (MPIRingTokenCommunication.cc:29-102);
 *   * communicateById_ (:365-410) -> allreduceRequests (MPIRingTokenCommunication.cc:105-157):
 *     one fp32 group, one plan (< 2^31-1 bytes, :495-546), executeCommunicatePlan_ (:548-733):
 *     memcpy every tensor into the fusion buffer, MPI_Allreduce(MPI_SUM) in place of
 *     MPICommunicator::allreduce (MPICommunicator.cc:14-28), memcpy back out, done() per tensor
 *     on the recv thread.
 * Timed as the SURVEY (§8d) prescribes: from the first handleRequest to the last done(), max over
 * ranks, best of `reps` after one warm-up.
 *
 * usage: mpiexec -n P ref_path_port <elements_per_tensor> <tensors> <reps>
 * prints (rank 0) one JSON line: {"P":..,"bytes":..,"best_ms":..,"mean_ms":..,"GiBs":..}
 */
#define _POSIX_C_SOURCE 200809L
#include <mpi.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

enum { TAG_META = 0, TAG_MSG = 1 };
enum { READY = 0, SYNC = 1, COMMUNICATE = 2, SHUT_DOWN = 3 };
enum { WAITING_TENSORS, WAITING_READY, WAITING_SYNC, WAITING_COMMUNICATE, COMMUNICATING };

typedef struct Token {
    unsigned char type;
    char *msg;
    size_t len;
    struct Token *next;
} Token;

static MPI_Comm comm;           /* the handler's communicator (a dup of the world) */
static int rank, P, ntens;
static size_t n;
static float **in, **out, *fin, *fout;
static char keyname[64];

/* registered requests (registeredRequest_), stage, parked READY key — under reg_mu */
static pthread_mutex_t reg_mu = PTHREAD_MUTEX_INITIALIZER;
static char *registered;        /* registered[t] */
static int nregistered, stage, waiting_ready = -1;
/* outgoing token queue (outputtingTokenQueue_) */
static pthread_mutex_t out_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t out_cv = PTHREAD_COND_INITIALIZER;
static Token *qhead, *qtail;
/* done() count of the current step */
static pthread_mutex_t done_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t done_cv = PTHREAD_COND_INITIALIZER;
static int ndone;
/* the reference's per-rank log file (Global.cc:10, GlobalLog.cc:43-49: each line written under a
   rwlock and flushed by std::endl); active by default for every communicated set
   (LogConfig.h:14, RingTokenCommunicateHandler.cc:365-410) and every op done (LogConfig.h:32,
   AllreduceOp.cc:55-56) */
static FILE *logf;
static pthread_mutex_t log_mu = PTHREAD_MUTEX_INITIALIZER;

static void log_line(const char *s) {
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    pthread_mutex_lock(&log_mu);
    fprintf(logf, "[INFO][TIME-%lld]: %s\n", (long long)ts.tv_sec * 1000 + ts.tv_nsec / 1000000, s);
    fflush(logf);
    pthread_mutex_unlock(&log_mu);
}

static void set_stage(int s) {
    pthread_mutex_lock(&reg_mu);
    stage = s;
    pthread_mutex_unlock(&reg_mu);
}

static const char *key_of(int t) {
    snprintf(keyname, sizeof keyname, "grad_%05d", t);
    return keyname;
}

static void enqueue(unsigned char type, const char *msg, size_t len) {
    Token *k = malloc(sizeof *k);
    k->type = type;
    k->msg = malloc(len + 1);
    memcpy(k->msg, msg, len);
    k->msg[len] = 0;
    k->len = len;
    k->next = NULL;
    pthread_mutex_lock(&out_mu);
    if (qtail) qtail->next = k; else qhead = k;
    qtail = k;
    pthread_cond_signal(&out_cv);
    pthread_mutex_unlock(&out_mu);
}

static void *send_main(void *arg) {
    int succ = (rank + 1) % P, stop = 0;
    (void)arg;
    while (!stop) {
        Token *k;
        pthread_mutex_lock(&out_mu);
        while (!qhead) pthread_cond_wait(&out_cv, &out_mu);
        k = qhead;
        qhead = NULL;
        qtail = NULL;
        pthread_mutex_unlock(&out_mu);
        while (k) {
            Token *nx = k->next;
            unsigned char meta[10];
            uint64_t l = k->len;
            meta[0] = k->type;
            meta[1] = 1; /* TOKEN_REQUEST_ALLREDUCE */
            memcpy(meta + 2, &l, 8);
            MPI_Send(meta, 10, MPI_BYTE, succ, TAG_META, comm);
            MPI_Send(k->msg, (int)k->len, MPI_CHAR, succ, TAG_MSG, comm);
            if (k->type == SHUT_DOWN) stop = 1;
            free(k->msg);
            free(k);
            k = nx;
        }
    }
    return NULL;
}

/* "Allreduce::grad_xxxxx\n" lines -> tensor indices (all keys are of that form here) */
static int parse_ids(const char *msg, int *ids) {
    int k = 0;
    const char *p = msg;
    while (*p) {
        const char *nl = strchr(p, '\n');
        const char *u = strstr(p, "::grad_");
        if (!nl) break;
        if (u && u < nl) ids[k++] = atoi(u + 7);
        p = nl + 1;
    }
    return k;
}

static size_t format_ids(const int *ids, int k, char *buf) {
    size_t len = 0;
    int i;
    for (i = 0; i < k; ++i) len += (size_t)sprintf(buf + len, "Allreduce::grad_%05d\n", ids[i]);
    return len;
}

static void communicate(const int *ids, int k) {
    int i;
    /* registered -> taken (communicateById_ erases them from the registry) */
    pthread_mutex_lock(&reg_mu);
    for (i = 0; i < k; ++i) {
        registered[ids[i]] = 0;
        --nregistered;
    }
    pthread_mutex_unlock(&reg_mu);
    {
        char desc[256];
        snprintf(desc, sizeof desc, "communicating Tensors: (%d x Allreduce::grad_*)", k);
        log_line(desc);
    }
    /* one fp32 plan: memcpy in, MPI_Allreduce, memcpy out, done() per request */
    for (i = 0; i < k; ++i) memcpy(fin + (size_t)i * n, in[ids[i]], n * 4);
    MPI_Allreduce(fin, fout, (int)(n * (size_t)k), MPI_FLOAT, MPI_SUM, comm);
    for (i = 0; i < k; ++i) {
        memcpy(out[ids[i]], fout + (size_t)i * n, n * 4);
        log_line("AllreduceOp done");
        pthread_mutex_lock(&done_mu);
        ++ndone;
        pthread_cond_signal(&done_cv);
        pthread_mutex_unlock(&done_mu);
    }
}

static void *recv_main(void *arg) {
    int pred = (rank + P - 1) % P;
    int *ids = malloc(sizeof(int) * (size_t)ntens), *keep = malloc(sizeof(int) * (size_t)ntens);
    char *buf = malloc((size_t)ntens * 40 + 64), *txt = malloc((size_t)ntens * 40 + 64);
    (void)arg;
    for (;;) {
        unsigned char meta[10];
        uint64_t l;
        int k, i, m;
        MPI_Recv(meta, 10, MPI_BYTE, pred, TAG_META, comm, MPI_STATUS_IGNORE);
        memcpy(&l, meta + 2, 8);
        MPI_Recv(buf, (int)l, MPI_CHAR, pred, TAG_MSG, comm, MPI_STATUS_IGNORE);
        buf[l] = 0;
        if (meta[0] == SHUT_DOWN) break;
        if (rank == 0) {  /* handleReceivingTokenAsTokenGenerator_ */
            if (meta[0] == READY) {
                pthread_mutex_lock(&reg_mu);
                for (k = 0, i = 0; i < ntens; ++i)
                    if (registered[i]) ids[k++] = i;
                stage = WAITING_SYNC;
                pthread_mutex_unlock(&reg_mu);
                enqueue(SYNC, txt, format_ids(ids, k, txt));
            } else if (meta[0] == SYNC) {
                set_stage(WAITING_COMMUNICATE);
                enqueue(COMMUNICATE, buf, l);
            } else if (meta[0] == COMMUNICATE) {
                set_stage(COMMUNICATING);
                k = parse_ids(buf, ids);
                communicate(ids, k);
                pthread_mutex_lock(&reg_mu);
                for (i = 0; i < ntens && !registered[i]; ++i) {
                }
                if (i < ntens) {
                    const char *key = key_of(i);
                    stage = WAITING_READY;
                    pthread_mutex_unlock(&reg_mu);
                    enqueue(READY, key, strlen(key));
                } else {
                    stage = WAITING_TENSORS;
                    pthread_mutex_unlock(&reg_mu);
                }
            }
        } else {  /* handleReceivingTokenAsTokenReceiver_ */
            if (meta[0] == READY) {
                const int t = atoi(buf + 5);  /* "grad_xxxxx" */
                pthread_mutex_lock(&reg_mu);
                if (registered[t]) {
                    stage = WAITING_SYNC;
                    pthread_mutex_unlock(&reg_mu);
                    enqueue(READY, buf, l);
                } else {
                    waiting_ready = t;  /* parked until handleRequest registers it */
                    stage = WAITING_TENSORS;
                    pthread_mutex_unlock(&reg_mu);
                }
            } else if (meta[0] == SYNC) {
                k = parse_ids(buf, ids);
                pthread_mutex_lock(&reg_mu);
                for (m = 0, i = 0; i < k; ++i)
                    if (registered[ids[i]]) keep[m++] = ids[i];
                stage = WAITING_COMMUNICATE;
                pthread_mutex_unlock(&reg_mu);
                enqueue(SYNC, txt, format_ids(keep, m, txt));
            } else if (meta[0] == COMMUNICATE) {
                set_stage(COMMUNICATING);
                enqueue(COMMUNICATE, buf, l);  /* forward first, then communicate */
                k = parse_ids(buf, ids);
                communicate(ids, k);
                set_stage(WAITING_READY);
            }
        }
    }
    free(ids);
    free(keep);
    free(buf);
    free(txt);
    return NULL;
}

/* handleRequest (RingTokenCommunicateHandler.cc:327-363) */
static void handle_request(int t) {
    pthread_mutex_lock(&reg_mu);
    registered[t] = 1;
    ++nregistered;
    if (rank == 0) {
        if (stage == WAITING_TENSORS) {
            stage = WAITING_READY;
            enqueue(READY, key_of(t), strlen(key_of(t)));
        }
    } else if (t == waiting_ready) {
        stage = WAITING_SYNC;
        waiting_ready = -1;
        enqueue(READY, key_of(t), strlen(key_of(t)));
    }
    pthread_mutex_unlock(&reg_mu);
}

int main(int argc, char **argv) {
    int provided, t, r, reps;
    double best = 1e30, sum = 0;
    pthread_t th_send, th_recv;
    MPI_Init_thread(&argc, &argv, MPI_THREAD_MULTIPLE, &provided); /* MPIBackend.cc:77-86 */
    if (provided < MPI_THREAD_MULTIPLE) {
        fprintf(stderr, "MPI_THREAD_MULTIPLE not provided\n");
        MPI_Abort(MPI_COMM_WORLD, 1);
    }
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &P);
    if (argc != 4 || P < 2) {
        if (!rank) fprintf(stderr, "usage: mpiexec -n P>=2 %s elements tensors reps\n", argv[0]);
        MPI_Abort(MPI_COMM_WORLD, 1);
    }
    MPI_Comm_dup(MPI_COMM_WORLD, &comm);
    {
        char path[512];
        const char *dir = getenv("TMPDIR");
        snprintf(path, sizeof path, "%s/ref_path_port-log-%d.txt", dir && *dir ? dir : "/tmp", rank);
        logf = fopen(path, "w");
        if (!logf) logf = fopen("/dev/null", "w");
    }
    n = (size_t)strtoull(argv[1], NULL, 10);
    ntens = atoi(argv[2]);
    reps = atoi(argv[3]);
    in = malloc(sizeof(float *) * (size_t)ntens);
    out = malloc(sizeof(float *) * (size_t)ntens);
    registered = calloc((size_t)ntens, 1);
    for (t = 0; t < ntens; ++t) {
        size_t i;
        in[t] = malloc(n * 4);
        out[t] = malloc(n * 4);
        for (i = 0; i < n; ++i) in[t][i] = (float)(rank + 1) * 0.5f + (float)(i % 7);
        memset(out[t], 0, n * 4);
    }
    fin = malloc(n * 4 * (size_t)ntens);
    fout = malloc(n * 4 * (size_t)ntens);
    memset(fin, 0, n * 4 * (size_t)ntens);
    memset(fout, 0, n * 4 * (size_t)ntens);
    stage = rank == 0 ? WAITING_TENSORS : WAITING_READY;
    pthread_create(&th_send, NULL, send_main, NULL);
    pthread_create(&th_recv, NULL, recv_main, NULL);
    for (r = -1; r < reps; ++r) { /* r = -1: warm-up */
        double t0, dt, mx;
        MPI_Barrier(MPI_COMM_WORLD);
        pthread_mutex_lock(&done_mu);
        ndone = 0;
        pthread_mutex_unlock(&done_mu);
        t0 = MPI_Wtime();
        for (t = 0; t < ntens; ++t) handle_request(t);  /* the TF ops' ComputeAsync calls */
        pthread_mutex_lock(&done_mu);
        while (ndone < ntens) pthread_cond_wait(&done_cv, &done_mu);
        pthread_mutex_unlock(&done_mu);
        dt = MPI_Wtime() - t0;
        MPI_Allreduce(&dt, &mx, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
        if (r >= 0) {
            sum += mx;
            if (mx < best) best = mx;
        }
    }
    /* ~RingTokenCommunicateHandler: every rank queues SHUT_DOWN, its successor's recv thread
       exits on it */
    MPI_Barrier(MPI_COMM_WORLD);
    enqueue(SHUT_DOWN, "shut down", 9);
    pthread_join(th_send, NULL);
    pthread_join(th_recv, NULL);
    if (rank == 0) {
        double bytes = (double)n * 4.0 * ntens;
        double expect0 = 0.5 * (double)P * (P + 1) / 2.0; /* element 0: sum of 0.5*(r+1) */
        printf("{\"P\": %d, \"bytes\": %.0f, \"tensors\": %d, \"best_ms\": %.4f, \"mean_ms\": %.4f, "
               "\"GiBs\": %.4f, \"threads_per_rank\": 3, \"check_out0\": %.3f, \"expect_out0\": %.3f}\n",
               P, bytes, ntens, best * 1e3, sum / reps * 1e3, bytes / best / 1073741824.0, out[0][0], expect0);
    }
    fclose(logf);
    MPI_Comm_free(&comm);
    MPI_Finalize();
    return 0;
}
