/*
 * ORACLE -- test infrastructure only.  Never linked into libigmhip.so; only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.
 *
 * fp64 CPU restatement of the reference M-step kernel: the LAMMPS run that
 * igm/model/kernel/lammps.py writes (create_lammps_data :63-146,
 * create_lammps_script :149-358) and executes (optimize :361-492), i.e.
 *
 *   units lj, mass 1, atom_style bond, boundary s s s
 *   pair_style soft (rc_ij = r_i + r_j, A_ij = ((r_i+r_j)/pi)^2 * evfactor;
 *       E = A [1 + cos(pi r / rc)], special_bonds 1 1 1 -> bonded pairs keep it)
 *                                                          lammps.py:117-137,179,189
 *   bond_style harmonic_upper_bound / harmonic_lower_bound (lammpgen; NOT in
 *       the container.  Restated as LAMMPS bond_harmonic: E = K (r - r0)^2 past
 *       the bound -- PARITY UNPINNED)      lammps.py:173-175
 *   fix ellipsoidalenvelope a b c k on all beads (lammpgen; energy form pinned
 *       by the demo summary's f_envelope0 for k > 0; force = -grad E)
 *                                                          lammps.py:292-303
 *   per stage: fix adapt (evf), velocity create (uniform, loop all, mom yes,
 *       Park-Miller RanPark, seed + stage), temp/rescale 1 T0 T1 0.1 1,
 *       nve/limit xmax, relax run first                    lammps.py:285-351
 *   min_style cg + minimize etol ftol maxiter maxeval (Polak-Ribiere, quadratic
 *       line search, dmax 0.1)                             lammps.py:354-356
 *   neighbor maxrad bin / neigh_modify every 1 check yes   lammps.py:216-219
 *
 * Also the M-step restraint assembly and scoring the GPU path replaces:
 *   oracle_hic_select   restraints/inter_hic.py:294-312 + intra_hic.py (f32 norm)
 *   oracle_violations   ModelingStep.py:511-557 + get_violation_histogram :859-869,
 *                       forces.py:131-139 (bond ratio), :222-247 (envelope scores)
 *
 * One structure per OpenMP thread, like the reference's one serial LAMMPS per
 * core (HPC_scripts/create_ipcluster_environment.sh); this is the CPU baseline.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/igm_hip.h"
#include "oracle_common.h"

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* ---------------------------------------------------------------- RanPark */
typedef struct {
    int seed;
} ranpark;
#define RP_IA 16807
#define RP_IM 2147483647
#define RP_AM (1.0 / RP_IM)
#define RP_IQ 127773
#define RP_IR 2836
static double rp_uniform(ranpark* r) {
    int k = r->seed / RP_IQ;
    r->seed = RP_IA * (r->seed - k * RP_IQ) - RP_IR * k;
    if (r->seed < 0) r->seed += RP_IM;
    return RP_AM * r->seed;
}

/* The reference prints np.float32 values with Python's shortest repr (e.g. the
 * PairIJ cutoff '561.4616' and the User radius '280.7308', lammps.py:135,146);
 * LAMMPS parses that decimal string as a double. */
static double f32_repr_double(float f) {
    char buf[64];
    for (int p = 1; p <= 9; ++p) {
        snprintf(buf, sizeof(buf), "%.*g", p, (double)f);
        if (strtof(buf, NULL) == f) return strtod(buf, NULL);
    }
    return (double)f;
}

/* memoised f32_repr_double (the cut-off of a pair only depends on f32(ri + rj)) */
typedef struct {
    uint32_t key[64];
    double val[64];
    int used[64];
} repr_cache;
static double repr_cached(repr_cache* c, float f) {
    uint32_t k;
    memcpy(&k, &f, 4);
    const int h = (int)((k * 2654435761u) >> 26);
    if (c->used[h] && c->key[h] == k) return c->val[h];
    c->used[h] = 1;
    c->key[h] = k;
    c->val[h] = f32_repr_double(f);
    return c->val[h];
}

/* ---------------------------------------------------------------- model */
typedef struct {
    repr_cache rc_cache;
    int n;               /* atoms */
    const float* radii;  /* per atom (f32, as the .hss holds them) */
    double* rlmp;        /* radius as LAMMPS reads it from the User section */
    const uint32_t* fl;  /* flags */
    int nb;              /* bonds */
    int* bi;
    int* bj;
    double* br0;
    double* bk;
    int* blow;
    const igm_mstep_params* prm;
    /* state */
    double *x, *v, *f;
    /* neighbour list (half, i < j by construction) */
    double* xlast;
    int* nb_start;
    int* nb_list;
    int nb_cap;
    double skin, cutmax;
    int nbuild;
    /* binning scratch */
    int* bin_head;
    int* bin_next;
    int nbins_cap;
    /* current factors */
    double evf, envf;
    /* energies of the last evaluation */
    double e_pair, e_bond, e_env[IGM_MAX_ENVELOPES];
} model_t;

static void build_neighbors(model_t* m) {
    const int n = m->n;
    double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
    int nbead = 0;
    for (int i = 0; i < n; ++i) {
        if (!(m->fl[i] & IGM_ATOM_BEAD)) continue;
        nbead++;
        for (int d = 0; d < 3; ++d) {
            if (m->x[3 * i + d] < lo[d]) lo[d] = m->x[3 * i + d];
            if (m->x[3 * i + d] > hi[d]) hi[d] = m->x[3 * i + d];
        }
    }
    const double cut = m->cutmax + m->skin;
    int nbin[3];
    double vol = 1.0;
    for (int d = 0; d < 3; ++d) vol *= (hi[d] - lo[d] > cut ? hi[d] - lo[d] : cut);
    double cs = cut;
    if (vol / (cs * cs * cs) > m->nbins_cap) cs = cbrt(vol / m->nbins_cap);
    for (int d = 0; d < 3; ++d) {
        nbin[d] = (int)floor((hi[d] - lo[d]) / cs);
        if (nbin[d] < 1) nbin[d] = 1;
    }
    const int ntot = nbin[0] * nbin[1] * nbin[2];
    for (int b = 0; b < ntot; ++b) m->bin_head[b] = -1;
    int* cellof = m->nb_start; /* temporary */
    /* insert in reverse index order so each bin list is ascending */
    for (int i = n - 1; i >= 0; --i) {
        if (!(m->fl[i] & IGM_ATOM_BEAD)) continue;
        int c[3];
        for (int d = 0; d < 3; ++d) {
            c[d] = (int)((m->x[3 * i + d] - lo[d]) / (hi[d] - lo[d] > 0 ? (hi[d] - lo[d]) : 1.0) * nbin[d]);
            if (c[d] >= nbin[d]) c[d] = nbin[d] - 1;
            if (c[d] < 0) c[d] = 0;
        }
        int b = (c[2] * nbin[1] + c[1]) * nbin[0] + c[0];
        cellof[i] = b;
        m->bin_next[i] = m->bin_head[b];
        m->bin_head[b] = i;
    }
    /* half list: j > i */
    int* start = (int*)malloc(sizeof(int) * (n + 1));
    int cnt = 0;
    const double cut2 = cut * cut;
    for (int i = 0; i < n; ++i) {
        start[i] = cnt;
        if (!(m->fl[i] & IGM_ATOM_BEAD)) continue;
        int b = cellof[i];
        int cx = b % nbin[0], cy = (b / nbin[0]) % nbin[1], cz = b / (nbin[0] * nbin[1]);
        for (int dz = -1; dz <= 1; ++dz)
            for (int dy = -1; dy <= 1; ++dy)
                for (int dx = -1; dx <= 1; ++dx) {
                    int x0 = cx + dx, y0 = cy + dy, z0 = cz + dz;
                    if (x0 < 0 || y0 < 0 || z0 < 0 || x0 >= nbin[0] || y0 >= nbin[1] || z0 >= nbin[2]) continue;
                    for (int j = m->bin_head[(z0 * nbin[1] + y0) * nbin[0] + x0]; j >= 0; j = m->bin_next[j]) {
                        if (j <= i) continue;
                        double ddx = m->x[3 * i] - m->x[3 * j], ddy = m->x[3 * i + 1] - m->x[3 * j + 1],
                               ddz = m->x[3 * i + 2] - m->x[3 * j + 2];
                        if (ddx * ddx + ddy * ddy + ddz * ddz < cut2) {
                            if (cnt >= m->nb_cap) {
                                m->nb_cap *= 2;
                                m->nb_list = (int*)realloc(m->nb_list, sizeof(int) * m->nb_cap);
                            }
                            m->nb_list[cnt++] = j;
                        }
                    }
                }
    }
    start[n] = cnt;
    memcpy(m->nb_start, start, sizeof(int) * (n + 1));
    free(start);
    memcpy(m->xlast, m->x, sizeof(double) * 3 * n);
    m->nbuild++;
    (void)nbead;
}

static void check_neighbors(model_t* m) {
    const double trig = 0.25 * m->skin * m->skin;
    for (int i = 0; i < m->n; ++i) {
        double dx = m->x[3 * i] - m->xlast[3 * i], dy = m->x[3 * i + 1] - m->xlast[3 * i + 1],
               dz = m->x[3 * i + 2] - m->xlast[3 * i + 2];
        if (dx * dx + dy * dy + dz * dz > trig) {
            build_neighbors(m);
            return;
        }
    }
}

/* E_env and its force on atom i for envelope e (k>0: outside, k<0: inside) */
static double envelope_atom(const model_t* m, int e, int i, double* fx, double* fy, double* fz) {
    const igm_mstep_params* p = m->prm;
    const double k = p->env_k[e];
    const double r = m->rlmp[i];
    double s[3];
    for (int d = 0; d < 3; ++d) s[d] = p->env_semiaxes[e][d] * m->envf - r; /* s2 = (abc - r)^2 */
    const double x = m->x[3 * i], y = m->x[3 * i + 1], z = m->x[3 * i + 2];
    const double k2 = x * x / (s[0] * s[0]) + y * y / (s[1] * s[1]) + z * z / (s[2] * s[2]);
    const int active = (k > 0) ? (k2 > 1.0) : (k2 < 1.0 && k2 > 0.0);
    if (!active) return 0.0;
    const double rn = sqrt(x * x + y * y + z * z);
    const double sk = sqrt(k2);
    const double t = (1.0 - 1.0 / sk) * rn;
    const double ka = fabs(k);
    /* dt/dx = (1 - k2^-1/2) x/|x| + |x| k2^-3/2 x/s^2 */
    const double a = (1.0 - 1.0 / sk) / rn;
    const double b = rn / (k2 * sk);
    *fx = -ka * t * (a * x + b * x / (s[0] * s[0]));
    *fy = -ka * t * (a * y + b * y / (s[1] * s[1]));
    *fz = -ka * t * (a * z + b * z / (s[2] * s[2]));
    return 0.5 * ka * t * t;
}

/* the volumetric map of IGM_ENV_VOLUME envelopes (one map for the whole call; the
 * form documented in include/igm_hip.h: pull a violating atom to the centre of its
 * voxel's nearest lamina voxel, E = |k|/2 d^2) */
static struct {
    int on, body, n[3];
    float origin[3], grid[3];
    const int32_t* vox;
} g_vol;

int oracle_set_volume(int body, const int32_t* n, const float* origin, const float* grid, const int32_t* vox) {
    g_vol.on = vox != NULL;
    g_vol.body = body;
    for (int d = 0; d < 3; ++d) {
        g_vol.n[d] = n ? n[d] : 0;
        g_vol.origin[d] = origin ? origin[d] : 0.0f;
        g_vol.grid[d] = grid ? grid[d] : 1.0f;
    }
    g_vol.vox = vox;
    return 0;
}

static double volume_atom(const model_t* m, int e, int i, double* fx, double* fy, double* fz) {
    const double k = m->prm->env_k[e];
    double o[3], g[3], t[3];
    int v[3];
    for (int d = 0; d < 3; ++d) {
        o[d] = (double)g_vol.origin[d] * m->envf;
        g[d] = (double)g_vol.grid[d] * m->envf;
        int iv = (int)rint((m->x[3 * i + d] - o[d]) / g[d]);
        v[d] = iv < 0 ? 0 : (iv >= g_vol.n[d] ? g_vol.n[d] - 1 : iv);
    }
    const int32_t* r = g_vol.vox + 4 * (((long)v[0] * g_vol.n[1] + v[1]) * g_vol.n[2] + v[2]);
    const int outside_ok = (g_vol.body == 0) == (k > 0);
    const int viol = outside_ok ? (r[3] == 0) : (r[3] != 0);
    if (!viol) return 0.0;
    for (int d = 0; d < 3; ++d) t[d] = m->x[3 * i + d] - (o[d] + g[d] * (double)r[d]);
    const double ka = fabs(k);
    *fx = -ka * t[0];
    *fy = -ka * t[1];
    *fz = -ka * t[2];
    return 0.5 * ka * (t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
}

static double energy_force(model_t* m) {
    check_neighbors(m);
    const int n = m->n;
    double* f = m->f;
    memset(f, 0, sizeof(double) * 3 * n);
    double ep = 0.0, eb = 0.0;
    /* pair soft */
    for (int i = 0; i < n; ++i) {
        const double ri = m->radii[i];
        for (int q = m->nb_start[i]; q < m->nb_start[i + 1]; ++q) {
            const int j = m->nb_list[q];
            const double dx = m->x[3 * i] - m->x[3 * j], dy = m->x[3 * i + 1] - m->x[3 * j + 1],
                         dz = m->x[3 * i + 2] - m->x[3 * j + 2];
            const double rsq = dx * dx + dy * dy + dz * dz;
            const float dc = (float)ri + m->radii[j]; /* dc = f32(ri + rj) */
            const double rc = repr_cached(&m->rc_cache, dc); /* PairIJ cutoff as printed */
            if (rsq >= rc * rc) continue;
            const double A = ((double)dc / M_PI) * ((double)dc / M_PI) * m->evf; /* A printed at full f64 */
            const double r = sqrt(rsq);
            const double arg = M_PI * r / rc;
            const double fpair = (r > 0.0) ? A * sin(arg) * M_PI / rc / r : 0.0;
            f[3 * i] += dx * fpair;
            f[3 * i + 1] += dy * fpair;
            f[3 * i + 2] += dz * fpair;
            f[3 * j] -= dx * fpair;
            f[3 * j + 1] -= dy * fpair;
            f[3 * j + 2] -= dz * fpair;
            ep += A * (1.0 + cos(arg));
        }
    }
    /* bonds */
    for (int b = 0; b < m->nb; ++b) {
        const int i = m->bi[b], j = m->bj[b];
        const double dx = m->x[3 * i] - m->x[3 * j], dy = m->x[3 * i + 1] - m->x[3 * j + 1],
                     dz = m->x[3 * i + 2] - m->x[3 * j + 2];
        const double r = sqrt(dx * dx + dy * dy + dz * dz);
        const double dr = r - m->br0[b];
        if (m->blow[b] ? (dr >= 0.0) : (dr <= 0.0)) continue;
        const double rk = m->bk[b] * dr;
        const double fb = (r > 0.0) ? -2.0 * rk / r : 0.0;
        f[3 * i] += dx * fb;
        f[3 * i + 1] += dy * fb;
        f[3 * i + 2] += dz * fb;
        f[3 * j] -= dx * fb;
        f[3 * j + 1] -= dy * fb;
        f[3 * j + 2] -= dz * fb;
        eb += rk * dr;
    }
    /* envelopes */
    double etot_env = 0.0;
    for (int e = 0; e < m->prm->nenvelopes; ++e) {
        double ee = 0.0;
        for (int i = 0; i < n; ++i) {
            if (!(m->fl[i] & (IGM_ATOM_ENV0 << e))) continue;
            double fx = 0, fy = 0, fz = 0;
            if (m->prm->env_kind[e] == IGM_ENV_VOLUME) {
                if (!g_vol.on) continue;
                ee += volume_atom(m, e, i, &fx, &fy, &fz);
            } else {
                ee += envelope_atom(m, e, i, &fx, &fy, &fz);
            }
            f[3 * i] += fx;
            f[3 * i + 1] += fy;
            f[3 * i + 2] += fz;
        }
        m->e_env[e] = ee;
        etot_env += ee;
    }
    /* fix setforce 0 on static dummies (lammps.py:222-223) */
    for (int i = 0; i < n; ++i)
        if (m->fl[i] & IGM_ATOM_FIXED) f[3 * i] = f[3 * i + 1] = f[3 * i + 2] = 0.0;
    m->e_pair = ep;
    m->e_bond = eb;
    return ep + eb + etot_env;
}

static int nonfixed_count(const model_t* m) {
    int c = 0;
    for (int i = 0; i < m->n; ++i) c += !(m->fl[i] & IGM_ATOM_FIXED);
    return c;
}

static double temperature(const model_t* m, int group_all) {
    double s = 0.0;
    int natom = 0;
    for (int i = 0; i < m->n; ++i) {
        if (!group_all && (m->fl[i] & IGM_ATOM_FIXED)) continue;
        natom++;
        s += m->v[3 * i] * m->v[3 * i] + m->v[3 * i + 1] * m->v[3 * i + 1] + m->v[3 * i + 2] * m->v[3 * i + 2];
    }
    const double dof = 3.0 * natom - 3.0;
    return dof > 0 ? s / dof : 0.0;
}

/* velocity nonfixed create T seed (dist uniform, loop all, mom yes) */
static void velocity_create(model_t* m, double t_desired, int seed) {
    ranpark rp = {seed};
    for (int i = 0; i < m->n; ++i) {
        double vx = rp_uniform(&rp) - 0.5;
        double vy = rp_uniform(&rp) - 0.5;
        double vz = rp_uniform(&rp) - 0.5;
        if (m->fl[i] & IGM_ATOM_FIXED) continue;
        m->v[3 * i] = vx;
        m->v[3 * i + 1] = vy;
        m->v[3 * i + 2] = vz;
    }
    double vcm[3] = {0, 0, 0};
    int cnt = 0;
    for (int i = 0; i < m->n; ++i) {
        if (m->fl[i] & IGM_ATOM_FIXED) continue;
        cnt++;
        for (int d = 0; d < 3; ++d) vcm[d] += m->v[3 * i + d];
    }
    for (int d = 0; d < 3; ++d) vcm[d] /= (cnt > 0 ? cnt : 1);
    for (int i = 0; i < m->n; ++i) {
        if (m->fl[i] & IGM_ATOM_FIXED) continue;
        for (int d = 0; d < 3; ++d) m->v[3 * i + d] -= vcm[d];
    }
    const double t = temperature(m, 0);
    const double factor = (t > 0.0) ? sqrt(t_desired / t) : 0.0;
    for (int i = 0; i < m->n; ++i) {
        if (m->fl[i] & IGM_ATOM_FIXED) continue;
        for (int d = 0; d < 3; ++d) m->v[3 * i + d] *= factor;
    }
}

/* run N steps: nve/limit + temp/rescale t0 -> t1 (Verlet: initial_integrate,
 * force, final_integrate, end_of_step) */
static void run_md(model_t* m, int nsteps, double t0, double t1, double xmax) {
    const igm_mstep_params* p = m->prm;
    const double dtv = p->timestep, dtf = 0.5 * p->timestep;
    const double vlimitsq = (xmax / dtv) * (xmax / dtv);
    const int n = m->n;
    energy_force(m); /* Verlet::setup */
    for (int step = 1; step <= nsteps; ++step) {
        for (int i = 0; i < n; ++i) {
            if (m->fl[i] & IGM_ATOM_FIXED) continue;
            double* v = m->v + 3 * i;
            const double* f = m->f + 3 * i;
            v[0] += dtf * f[0];
            v[1] += dtf * f[1];
            v[2] += dtf * f[2];
            const double vsq = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
            if (vsq > vlimitsq) {
                const double s = sqrt(vlimitsq / vsq);
                v[0] *= s;
                v[1] *= s;
                v[2] *= s;
            }
            m->x[3 * i] += dtv * v[0];
            m->x[3 * i + 1] += dtv * v[1];
            m->x[3 * i + 2] += dtv * v[2];
        }
        energy_force(m);
        for (int i = 0; i < n; ++i) {
            if (m->fl[i] & IGM_ATOM_FIXED) continue;
            double* v = m->v + 3 * i;
            const double* f = m->f + 3 * i;
            v[0] += dtf * f[0];
            v[1] += dtf * f[1];
            v[2] += dtf * f[2];
            const double vsq = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
            if (vsq > vlimitsq) {
                const double s = sqrt(vlimitsq / vsq);
                v[0] *= s;
                v[1] *= s;
                v[2] *= s;
            }
        }
        /* fix temp/rescale 1 t0 t1 window fraction */
        const double tcur = temperature(m, 0);
        if (tcur > 0.0) {
            const double delta = (double)step / (double)nsteps;
            double tt = t0 + delta * (t1 - t0);
            if (fabs(tcur - tt) > p->t_window) {
                tt = tcur - p->t_fraction * (tcur - tt);
                const double factor = sqrt(tt / tcur);
                for (int i = 0; i < n; ++i) {
                    if (m->fl[i] & IGM_ATOM_FIXED) continue;
                    m->v[3 * i] *= factor;
                    m->v[3 * i + 1] *= factor;
                    m->v[3 * i + 2] *= factor;
                }
            }
        }
    }
}

/* ---------------------------------------------------------------- CG */
enum { MAXITER = 1, MAXEVAL, ETOL, FTOL, DOWNHILL, ZEROALPHA, ZEROFORCE, ZEROQUAD };
#define ALPHA_MAX 1.0
#define ALPHA_REDUCE 0.5
#define BACKTRACK_SLOPE 0.4
#define QUADRATIC_TOL 0.1
#define EMACH 1.0e-8
#define EPS_QUAD 1.0e-28
#define EPS_ENERGY 1.0e-8

typedef struct {
    double *x0, *g, *h;
    int neval;
    double ecurrent;
} cgstate;

static double alpha_step(model_t* m, cgstate* cs, double alpha) {
    const int n3 = 3 * m->n;
    for (int i = 0; i < n3; ++i) m->x[i] = cs->x0[i];
    if (alpha > 0.0)
        for (int i = 0; i < n3; ++i) m->x[i] += alpha * cs->h[i];
    cs->neval++;
    return energy_force(m);
}

static int linemin_quadratic(model_t* m, cgstate* cs, double eoriginal, double* alpha_out) {
    const int n3 = 3 * m->n;
    double fdothall = 0.0;
    for (int i = 0; i < n3; ++i) fdothall += m->f[i] * cs->h[i];
    if (fdothall <= 0.0) return DOWNHILL;
    double hmaxall = 0.0;
    for (int i = 0; i < n3; ++i)
        if (fabs(cs->h[i]) > hmaxall) hmaxall = fabs(cs->h[i]);
    if (hmaxall == 0.0) return ZEROFORCE;
    double alphamax = m->prm->dmax / hmaxall;
    if (alphamax > ALPHA_MAX) alphamax = ALPHA_MAX;
    for (int i = 0; i < n3; ++i) cs->x0[i] = m->x[i];
    double alpha = alphamax, engprev = eoriginal, alphaprev = 0.0, fhprev = fdothall;
    for (;;) {
        cs->ecurrent = alpha_step(m, cs, alpha);
        double ff = 0.0, fh = 0.0;
        for (int i = 0; i < n3; ++i) {
            ff += m->f[i] * m->f[i];
            fh += m->f[i] * cs->h[i];
        }
        (void)ff;
        const double delfh = fh - fhprev;
        if (fabs(fh) < EPS_QUAD || fabs(delfh) < EPS_QUAD) {
            cs->ecurrent = alpha_step(m, cs, 0.0);
            return ZEROQUAD;
        }
        const double relerr = fabs(1.0 - (0.5 * (alpha - alphaprev) * (fh + fhprev) + cs->ecurrent) / engprev);
        const double alpha0 = alpha - (alpha - alphaprev) * fh / delfh;
        if (relerr <= QUADRATIC_TOL && alpha0 > 0.0 && alpha0 < alphamax) {
            cs->ecurrent = alpha_step(m, cs, alpha0);
            if (cs->ecurrent - eoriginal < EMACH) {
                *alpha_out = alpha0;
                return 0;
            }
        }
        const double de_ideal = -BACKTRACK_SLOPE * alpha * fdothall;
        const double de = cs->ecurrent - eoriginal;
        if (de <= de_ideal) {
            *alpha_out = alpha;
            return 0;
        }
        fhprev = fh;
        engprev = cs->ecurrent;
        alphaprev = alpha;
        alpha *= ALPHA_REDUCE;
        if (alpha <= 0.0 || de_ideal >= -EMACH) {
            cs->ecurrent = alpha_step(m, cs, 0.0);
            return ZEROALPHA;
        }
    }
}

static int minimize_cg(model_t* m, igm_opt_info* info) {
    const igm_mstep_params* p = m->prm;
    const int n3 = 3 * m->n;
    cgstate cs;
    cs.x0 = (double*)calloc(n3, sizeof(double));
    cs.g = (double*)calloc(n3, sizeof(double));
    cs.h = (double*)calloc(n3, sizeof(double));
    cs.neval = 0;
    cs.ecurrent = energy_force(m); /* Min::setup */
    info->einitial = cs.ecurrent;
    for (int i = 0; i < n3; ++i) cs.h[i] = cs.g[i] = m->f[i];
    double gg = 0.0;
    for (int i = 0; i < n3; ++i) gg += m->f[i] * m->f[i];
    int stop = MAXITER, niter = 0;
    const int nlimit = n3;
    for (int iter = 0; iter < p->max_cg_iter; ++iter) {
        niter++;
        const double eprevious = cs.ecurrent;
        double alpha = 0.0;
        int fail = linemin_quadratic(m, &cs, cs.ecurrent, &alpha);
        if (fail) {
            stop = fail;
            break;
        }
        if (cs.neval >= p->max_cg_eval) {
            stop = MAXEVAL;
            break;
        }
        if (fabs(cs.ecurrent - eprevious) <
            p->etol * 0.5 * (fabs(cs.ecurrent) + fabs(eprevious) + EPS_ENERGY)) {
            stop = ETOL;
            break;
        }
        double d0 = 0.0, d1 = 0.0;
        for (int i = 0; i < n3; ++i) {
            d0 += m->f[i] * m->f[i];
            d1 += m->f[i] * cs.g[i];
        }
        if (p->ftol > 0.0 && d0 < p->ftol * p->ftol) {
            stop = FTOL;
            break;
        }
        double beta = (d0 - d1) / gg;
        if (beta < 0.0) beta = 0.0;
        if ((niter + 1) % nlimit == 0) beta = 0.0;
        gg = d0;
        double gh = 0.0;
        for (int i = 0; i < n3; ++i) {
            cs.g[i] = m->f[i];
            cs.h[i] = cs.g[i] + beta * cs.h[i];
            gh += cs.g[i] * cs.h[i];
        }
        if (gh <= 0.0)
            for (int i = 0; i < n3; ++i) cs.h[i] = cs.g[i];
    }
    /* Min::run: energy at the final state for the last thermo output */
    double fn = 0.0;
    for (int i = 0; i < n3; ++i) fn += m->f[i] * m->f[i];
    info->fnorm_final = sqrt(fn);
    info->final_energy = cs.ecurrent;
    info->cg_iters = niter;
    info->cg_evals = cs.neval;
    info->stop_reason = stop;
    free(cs.x0);
    free(cs.g);
    free(cs.h);
    return 0;
}

/* ---------------------------------------------------------------- setup */
static void model_init(model_t* m, const igm_mstep_params* prm, int natom, const float* xyz, const float* radii,
                       const uint32_t* fl, const igm_bond* shared, int64_t nshared, const igm_bond* own,
                       int64_t nown) {
    memset(m, 0, sizeof(*m));
    m->n = natom;
    m->radii = radii;
    m->fl = fl;
    m->prm = prm;
    m->nb = (int)(nshared + nown);
    m->bi = (int*)malloc(sizeof(int) * (m->nb + 1));
    m->bj = (int*)malloc(sizeof(int) * (m->nb + 1));
    m->br0 = (double*)malloc(sizeof(double) * (m->nb + 1));
    m->bk = (double*)malloc(sizeof(double) * (m->nb + 1));
    m->blow = (int*)malloc(sizeof(int) * (m->nb + 1));
    for (int64_t b = 0; b < nshared + nown; ++b) {
        const igm_bond* bd = (b < nshared) ? &shared[b] : &own[b - nshared];
        m->bi[b] = (int)bd->i;
        m->bj[b] = (int)(bd->j & 0x7fffffffu);
        m->blow[b] = (bd->j >> 31) & 1u;
        m->br0[b] = bd->r0;
        m->bk[b] = bd->k;
    }
    m->rlmp = (double*)malloc(sizeof(double) * natom);
    for (int i = 0; i < natom; ++i) m->rlmp[i] = f32_repr_double(radii[i]);
    m->x = (double*)malloc(sizeof(double) * 3 * natom);
    m->v = (double*)calloc(3 * natom, sizeof(double));
    m->f = (double*)calloc(3 * natom, sizeof(double));
    m->xlast = (double*)malloc(sizeof(double) * 3 * natom);
    for (int i = 0; i < 3 * natom; ++i) m->x[i] = xyz[i];
    double rmax = 0.0;
    for (int i = 0; i < natom; ++i)
        if ((fl[i] & IGM_ATOM_BEAD) && radii[i] > rmax) rmax = radii[i];
    m->cutmax = 2.0 * rmax;
    m->skin = prm->skin > 0 ? prm->skin : rmax;
    m->nb_start = (int*)malloc(sizeof(int) * (natom + 1));
    m->nb_cap = 64 * natom + 64;
    m->nb_list = (int*)malloc(sizeof(int) * m->nb_cap);
    m->nbins_cap = 8 * natom + 64;
    m->bin_head = (int*)malloc(sizeof(int) * m->nbins_cap);
    m->bin_next = (int*)malloc(sizeof(int) * natom);
    m->evf = prm->evfactor_base;
    m->envf = 1.0;
    build_neighbors(m);
}

static void model_free(model_t* m) {
    free(m->bi);
    free(m->bj);
    free(m->br0);
    free(m->bk);
    free(m->blow);
    free(m->rlmp);
    free(m->x);
    free(m->v);
    free(m->f);
    free(m->xlast);
    free(m->nb_start);
    free(m->nb_list);
    free(m->bin_head);
    free(m->bin_next);
}

static void fill_info_thermo(model_t* m, igm_opt_info* info) {
    info->pair_energy = m->e_pair;
    info->bond_energy = m->e_bond;
    for (int e = 0; e < IGM_MAX_ENVELOPES; ++e) info->env_energy[e] = (e < m->prm->nenvelopes) ? m->e_env[e] : 0.0;
    info->temp = temperature(m, 1); /* thermo temp: group all */
    info->nrebuild = m->nbuild;
}

/* the whole M-step protocol for one structure (fp64) */
static void run_one(const igm_mstep_params* p, int natom, float* xyz, const float* radii, const uint32_t* fl,
                    const igm_bond* shared, int64_t nshared, const igm_bond* own, int64_t nown, int seed,
                    igm_opt_info* info, double* xout) {
    model_t m;
    model_init(&m, p, natom, xyz, radii, fl, shared, nshared, own, nown);
    for (int k = 0; k < p->nstages; ++k) {
        m.evf = p->evfactor_base * p->evfactor[k]; /* fix adapt ... scale yes */
        m.envf = p->envfactor[k];
        if (p->relax_steps > 0) {
            velocity_create(&m, p->relax_temperature, seed + k);
            run_md(&m, p->relax_steps, p->relax_temperature, p->relax_temperature, p->relax_max_velocity);
        }
        velocity_create(&m, p->tstart[k], seed + k);
        run_md(&m, p->mdsteps[k], p->tstart[k], p->tstop[k], p->max_velocity);
    }
    /* unfix adapt (reset yes): original prefactor; the last envelope fix stays */
    m.evf = p->evfactor_base;
    if (p->nstages > 0) m.envf = p->envfactor[p->nstages - 1];
    minimize_cg(&m, info);
    fill_info_thermo(&m, info);
    for (int i = 0; i < 3 * natom; ++i) xyz[i] = (float)m.x[i];
    if (xout) memcpy(xout, m.x, sizeof(double) * 3 * natom);
    model_free(&m);
}

/* fl_stride: 0 = one flag row shared by every structure, natom = a row per structure
 * (the GPU's IGM_MSTEP_STRUCT_FLAGS: DamID envelope members, SPRITE centroid slots) */
int oracle_mstep_run_sf(const igm_mstep_params* p, int32_t nstruct, int32_t natom, float* xyz, const float* radii,
                        const uint32_t* fl, int64_t fl_stride, const igm_bond* shared, int64_t nshared,
                        const int64_t* sptr, const igm_bond* sbonds, const int32_t* seeds, igm_opt_info* info,
                        double* xout, int32_t nthreads) {
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
    for (int s = 0; s < nstruct; ++s) {
        const int64_t b0 = sptr ? sptr[s] : 0, b1 = sptr ? sptr[s + 1] : 0;
        run_one(p, natom, xyz + (size_t)s * natom * 3, radii, fl + (size_t)s * fl_stride, shared, nshared,
                sbonds + b0, b1 - b0, seeds[s], &info[s], xout ? xout + (size_t)s * natom * 3 : NULL);
    }
    return 0;
}

int oracle_mstep_run(const igm_mstep_params* p, int32_t nstruct, int32_t natom, float* xyz, const float* radii,
                     const uint32_t* fl, const igm_bond* shared, int64_t nshared, const int64_t* sptr,
                     const igm_bond* sbonds, const int32_t* seeds, igm_opt_info* info, double* xout,
                     int32_t nthreads) {
    return oracle_mstep_run_sf(p, nstruct, natom, xyz, radii, fl, 0, shared, nshared, sptr, sbonds, seeds, info, xout,
                               nthreads);
}

/* forces (f64) and energies {total, pair, bond, env0..3} */
int oracle_mstep_forces(const igm_mstep_params* p, int32_t nstruct, int32_t natom, const float* xyz,
                        const float* radii, const uint32_t* fl, const igm_bond* shared, int64_t nshared,
                        const int64_t* sptr, const igm_bond* sbonds, double evf, double envf, double* forces,
                        double* energies) {
    for (int s = 0; s < nstruct; ++s) {
        model_t m;
        const int64_t b0 = sptr ? sptr[s] : 0, b1 = sptr ? sptr[s + 1] : 0;
        model_init(&m, p, natom, xyz + (size_t)s * natom * 3, radii, fl, shared, nshared, sbonds + b0, b1 - b0);
        m.evf = evf;
        m.envf = envf;
        const double e = energy_force(&m);
        memcpy(forces + (size_t)s * natom * 3, m.f, sizeof(double) * 3 * natom);
        double* en = energies + (size_t)s * (3 + IGM_MAX_ENVELOPES);
        en[0] = e;
        en[1] = m.e_pair;
        en[2] = m.e_bond;
        for (int k = 0; k < IGM_MAX_ENVELOPES; ++k) en[3 + k] = k < p->nenvelopes ? m.e_env[k] : 0.0;
        model_free(&m);
    }
    return 0;
}

/* short MD segment from given x, v (f64 in/out) */
int oracle_mstep_md(const igm_mstep_params* p, int32_t nstruct, int32_t natom, double* x, double* v,
                    const float* radii, const uint32_t* fl, const igm_bond* shared, int64_t nshared,
                    const int64_t* sptr, const igm_bond* sbonds, double evf, double envf, double t0, double t1,
                    double xmax, int32_t nsteps, int32_t nthreads) {
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
    for (int s = 0; s < nstruct; ++s) {
        float* xf = (float*)malloc(sizeof(float) * 3 * natom);
        model_t m;
        const int64_t b0 = sptr ? sptr[s] : 0, b1 = sptr ? sptr[s + 1] : 0;
        for (int i = 0; i < 3 * natom; ++i) xf[i] = (float)x[(size_t)s * natom * 3 + i];
        model_init(&m, p, natom, xf, radii, fl, shared, nshared, sbonds + b0, b1 - b0);
        memcpy(m.x, x + (size_t)s * natom * 3, sizeof(double) * 3 * natom);
        build_neighbors(&m);
        memcpy(m.v, v + (size_t)s * natom * 3, sizeof(double) * 3 * natom);
        m.evf = evf;
        m.envf = envf;
        run_md(&m, nsteps, t0, t1, xmax);
        memcpy(x + (size_t)s * natom * 3, m.x, sizeof(double) * 3 * natom);
        memcpy(v + (size_t)s * natom * 3, m.v, sizeof(double) * 3 * natom);
        model_free(&m);
        free(xf);
    }
    return 0;
}

/* velocity create only (for RNG-stream parity tests) */
int oracle_velocity_create(int32_t natom, const uint32_t* fl, double t_desired, int32_t seed, double* v) {
    model_t m;
    memset(&m, 0, sizeof(m));
    m.n = natom;
    m.fl = fl;
    m.v = v;
    velocity_create(&m, t_desired, seed);
    return 0;
}

/* Hi-C restraint selection for structure-major xyz (nstruct, natom, 3):
 * ||x_i - x_j|| computed in f32 exactly as numpy's norm of a 3-vector
 * (sqrt(fl32(fl32(dx^2 + dy^2) + dz^2)), particle.py:35-36) compared with
 * the f32 activation distance; inter rows first, then intra (ModelingStep.py:392-398).
 * out_sel: (nstruct, n_act) uint8: 1 = inter bond, 2 = intra bond, 0 = none. */
int oracle_hic_select(int32_t nstruct, int32_t natom, const float* xyz, const int32_t* chrom, const int32_t* row,
                      const int32_t* col, const float* dist, int64_t n_act, uint8_t* out_sel) {
    for (int s = 0; s < nstruct; ++s) {
        const float* x = xyz + (size_t)s * natom * 3;
        for (int64_t q = 0; q < n_act; ++q) {
            const int i = row[q], j = col[q];
            const float dx = x[3 * i] - x[3 * j], dy = x[3 * i + 1] - x[3 * j + 1], dz = x[3 * i + 2] - x[3 * j + 2];
            const float d = sqrtf((dx * dx + dy * dy) + dz * dz);
            uint8_t sel = 0;
            if (d <= dist[q]) sel = (chrom[i] != chrom[j]) ? 1 : 2;
            out_sel[(size_t)s * n_act + q] = sel;
        }
    }
    return 0;
}

/* n-th uniform() of RanPark(seed) (1-based), serial -- known-answer test hook */
double oracle_ranpark_nth(int32_t seed, int64_t n) {
    ranpark rp = {seed};
    double u = 0.0;
    for (int64_t k = 0; k < n; ++k) u = rp_uniform(&rp);
    return u;
}
int32_t oracle_ranpark_state(int32_t seed, int64_t n) {
    ranpark rp = {seed};
    for (int64_t k = 0; k < n; ++k) rp_uniform(&rp);
    return rp.seed;
}
