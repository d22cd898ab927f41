/*
 * oracle/mpi_allreduce_driver.c — TEST INFRASTRUCTURE ONLY (golden-vector generator).
 *
 * Calls MPICH's MPI_Allreduce exactly as the reference's data plane does
 * (src/cpp/communicate/backend/mpi/MPICommunicator.cc:14-28: one call, MPI_SUM, count =
 * elements, datatype from MPIBackend::DataType2MPIType, MPIBackend.cc:48-66), under
 * MPI_THREAD_MULTIPLE (MPIBackend.cc:77-86). It is our own driver around the third-party
 * MPICH 3.3.2 shipped in the image (/opt/conda), not reference source.
 *
 * usage: mpiexec -n P mpi_allreduce_driver <dtype> <elements> <dir>
 *   reads <dir>/in_<rank>.bin, writes <dir>/out_<rank>.bin
 */
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>

static MPI_Datatype to_mpi(int dt, size_t *es) {
    switch (dt) {
        case 1: *es = 4; return MPI_FLOAT;      /* DT_FLOAT  */
        case 2: *es = 8; return MPI_DOUBLE;     /* DT_DOUBLE */
        case 3: *es = 4; return MPI_INT;        /* DT_INT32  */
        case 9: *es = 8; return MPI_INT64_T;    /* DT_INT64  */
        case 23: *es = 8; return MPI_UINT64_T;  /* DT_UINT64 */
        default: *es = 0; return MPI_DATATYPE_NULL;
    }
}

int main(int argc, char **argv) {
    int provided, rank, size, dt;
    size_t n, es, got;
    char path[4096];
    void *in, *out;
    FILE *f;
    MPI_Datatype t;
    MPI_Init_thread(&argc, &argv, MPI_THREAD_MULTIPLE, &provided);
    if (argc != 4) { fprintf(stderr, "usage: %s dtype elements dir\n", argv[0]); MPI_Abort(MPI_COMM_WORLD, 2); }
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &size);
    dt = atoi(argv[1]);
    n = (size_t)strtoull(argv[2], NULL, 10);
    t = to_mpi(dt, &es);
    if (!es) { fprintf(stderr, "unsupported dtype %d\n", dt); MPI_Abort(MPI_COMM_WORLD, 3); }
    in = malloc(n * es + 1);
    out = malloc(n * es + 1);
    snprintf(path, sizeof path, "%s/in_%d.bin", argv[3], rank);
    f = fopen(path, "rb");
    if (!f) { perror(path); MPI_Abort(MPI_COMM_WORLD, 4); }
    got = fread(in, es, n, f);
    fclose(f);
    if (got != n) { fprintf(stderr, "short read %s\n", path); MPI_Abort(MPI_COMM_WORLD, 5); }
    MPI_Allreduce(in, out, (int)n, t, MPI_SUM, MPI_COMM_WORLD);
    snprintf(path, sizeof path, "%s/out_%d.bin", argv[3], rank);
    f = fopen(path, "wb");
    if (!f) { perror(path); MPI_Abort(MPI_COMM_WORLD, 6); }
    fwrite(out, es, n, f);
    fclose(f);
    free(in);
    free(out);
    MPI_Finalize();
    return 0;
}
