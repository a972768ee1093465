/*
 * CPU restatement (OpenMP, plain C) of trex's Sankoff forward + gradient.
 * TEST INFRASTRUCTURE / CPU BASELINE ONLY: called by tests/ (as a checker) and
 * by bench.py's cpu_baseline leg (as the timed CPU reference).  Never linked
 * into libtrexhip.so.
 *
 * Follows the reference recurrence directly, in node-index order like
 * run_dp's fori_loop (maraxen/trex src/trex/sankoff.py:87-92) with its child
 * rules (sankoff.py:60,67: -1 fill or c >= node reads the 1e5 row,
 * c < n_leaves is a leaf row initialised at :49-52), vectorised over a block
 * of sites the way vectorized_dp vmaps over sites (:97).  tau == 0 is the
 * hard min (:68) with JAX's tie-averaged min gradient; tau > 0 the softmin
 * relaxation of DESIGN.md, in the per-row stabilised form (no factoring).
 *
 * Two instantiations of one body (cpu_port_impl.h), in two translation
 * units with their own flags (oracle/Makefile):
 *   sankoff_cpu_fwd_bwd    (this file) fp32 arithmetic, as trex computes --
 *                          the timed CPU baseline ("port"), built with
 *                          -ffast-math so its exp / log vectorise (glibc's
 *                          vector math needs it); every sentinel is finite
 *                          (1e5, FLT_MAX), so finite-math is sound here;
 *   sankoff_cpu64_fwd_bwd  (cpu_port64.c) fp64 arithmetic, strict IEEE --
 *                          the checker for GPU results at sizes the numpy
 *                          oracle cannot hold (C4's 1024-tree batch).
 * Both are pinned to oracle/softmin_ref.py by tests/test_cpu_port_cpu.py.
 */
#include <float.h>
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define BLK 64
#define SENT 1e5

#define REAL float
#define REAL_BIG FLT_MAX
#define EXP expf
#define LOG logf
#define FN sankoff_cpu_fwd_bwd
#define NM(x) x##_f32
#include "cpu_port_impl.h"
