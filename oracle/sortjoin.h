/* sortjoin.h -- CPU BASELINE / TEST INFRASTRUCTURE ONLY (see sortjoin.c). */
#ifndef SORTJOIN_H
#define SORTJOIN_H

#include <stddef.h>
#include <stdint.h>

typedef struct sj_window sj_window;

/* Marshalled probes, the layout comdb2_amd's marshaller emits
 * (hsc_marshalled in include/hip_serial.h): key words SoA [W][n]. */
typedef struct sj_probes {
    size_t n;
    const uint64_t *lo, *hi;
    const uint32_t *gid;
    const uint64_t *snap;
    const uint32_t *txn;
    size_t n_lock;
    const uint32_t *lock_table;
    const uint64_t *lock_snap;
    const uint32_t *lock_txn;
    const uint64_t *table_max;  /* [ntables] max commit LSN per table */
    uint32_t ntables;
} sj_probes;

/* rows: gid[n], words [W][n] (big-endian key words), lsn[n]; any order */
sj_window *sj_build(size_t n, int W, uint32_t ngroups, const uint32_t *gid,
                    const uint64_t *words, const uint64_t *lsn, double *secs);
void sj_free(sj_window *w);
size_t sj_rows(const sj_window *w);
/* ORs the join verdicts into verdict[n_txn]; returns wall seconds */
double sj_probe(const sj_window *w, const sj_probes *p, int nthreads, uint8_t *verdict);

#endif
