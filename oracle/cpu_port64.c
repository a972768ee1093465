/*
 * fp64 instantiation of the OpenMP C restatement (see cpu_port.c): the
 * checker for full-batch GPU runs.  TEST INFRASTRUCTURE ONLY.  Built with
 * strict IEEE flags (no -ffast-math): oracle/Makefile.
 */
#include <float.h>
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define BLK 64
#define SENT 1e5

#define REAL double
#define REAL_BIG DBL_MAX
#define EXP exp
#define LOG log
#define FN sankoff_cpu64_fwd_bwd
#define NM(x) x##_f64
#include "cpu_port_impl.h"
