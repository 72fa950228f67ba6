/*
 * igm_hip.h -- C ABI of libigmhip.so, the MI355X (gfx950) engine that replaces
 * the two hot paths of IGM (bonimba87/igm):
 *
 *   A-step  ActivationDistanceStep.get_actdist  (igm/steps/ActivationDistanceStep.py:336-485)
 *           applied to every kept haploid pair   (ActivationDistanceStep.py:196-230)
 *   M-step  serial-LAMMPS anneal + CG per structure, i.e. lammps.optimize
 *           (igm/model/kernel/lammps.py:361-492) driven by ModelingStep.task
 *           (igm/steps/ModelingStep.py:164-573), batched over the population.
 *
 * Plain C types only (no torch types).  Every entry point returns IGM_OK (0) or
 * a negative IGM_E_* code; igm_last_error() then holds a message.  The Python
 * shim maps a nonzero code to RuntimeError(message), which is the reference's
 * behaviour on a failed LAMMPS run (lammps.py:453-457).
 *
 * Ownership: the caller owns every buffer.  With IGM_DEVICE_PTRS set in `flags`
 * all array arguments are device pointers on the context's device (e.g. torch
 * tensors' data_ptr()); otherwise they are host pointers and the library stages
 * them.  Calls are stream-ordered on the context stream and return after the
 * work has completed unless IGM_ASYNC is set (device-pointer mode only).
 * Threading: one igm_ctx per (host thread, GPU); a context is not thread safe.
 */
#ifndef IGM_HIP_H
#define IGM_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IGM_OK 0
#define IGM_E_INVALID (-1)     /* bad argument                              */
#define IGM_E_HIP (-2)         /* HIP runtime error                         */
#define IGM_E_NOMEM (-3)       /* device allocation failed                  */
#define IGM_E_OVERFLOW (-4)    /* neighbour list / row capacity exceeded    */
#define IGM_E_UNSUPPORTED (-5) /* size outside the implemented envelope      */

#define IGM_DEVICE_PTRS 0x1u /* array arguments are device pointers        */
#define IGM_ASYNC 0x2u       /* do not synchronise before returning        */
#define IGM_F32_PATH 0x4u    /* igm_mstep_forces: use the f32 MD force path */

typedef struct igm_ctx igm_ctx;

/* ---- context ------------------------------------------------------------- */
int igm_ctx_create(int device, igm_ctx** out);
void igm_ctx_destroy(igm_ctx* ctx);
const char* igm_last_error(const igm_ctx* ctx);
/* Use an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream);
 * NULL restores the context's own stream. */
int igm_ctx_set_stream(igm_ctx* ctx, void* hip_stream);
int igm_ctx_synchronize(igm_ctx* ctx);
/* Milliseconds of the last launch of the named kernel family measured with
 * HIP events on the context stream ("actdist", "anneal", "hic_select", ...). */
double igm_last_kernel_ms(const igm_ctx* ctx, const char* name);
const char* igm_version(void);

/* ---- A-step: activation distances ------------------------------------------
 * Replaces the per-pair loop ActivationDistanceStep.task (py:215-222) and
 * get_actdist (py:336-485) over the WHOLE kept-pair list in one call, and the
 * text round trip of task/reduce (py:228-230, 249): the emitted dist/prob are
 * float32(float('%10.4f' % ad)) and float32(float('%.4f' % p)), bit-exact.
 */
typedef struct {
    int32_t i, j;  /* haploid loci, i != j expected (i == j -> no rows)  */
    double pwish;  /* target probability (hcs value, f32 widened)        */
    double plast;  /* previous iteration's corrected probability         */
} igm_pair;        /* 24 bytes: the row layout of the reference '<b>.in.npy' batches */

typedef struct {
    int32_t row, col; /* diploid bead indices                                */
    float dist, prob; /* actdist.hdf5 {row i4, col i4, dist f4, prob f4}     */
} igm_actdist_row;

typedef struct {
    double ad;     /* sqrt of the o-th smallest d^2 (f64), NaN if no rows */
    double p;      /* corrected probability used (f64)                    */
    double pnow;   /* count(d^2 <= rcut^2) / (n*S)                        */
    int32_t o;     /* order statistic index, -1 if no rows                */
    int32_t nrows; /* rows emitted for this pair (0, 1, 2 or 4 ...)       */
} igm_pair_result;

int igm_astep_actdist(igm_ctx* ctx, uint32_t flags,
                      const float* xyz, /* bead-major (nbead, nstruct, 3) f32, the .hss layout */
                      int32_t nbead, int32_t nstruct,
                      const float* radii,     /* (nbead)                                      */
                      const int32_t* copy_ptr, /* (nhap+1) CSR of index.copy_index             */
                      const int32_t* copy_idx, /* diploid bead ids                             */
                      int32_t nhap,
                      const int32_t* chrom, /* chrom[i] as the reference indexes it (hss index.chrom) */
                      const igm_pair* pairs, int64_t npairs,
                      double contact_range, int32_t it_corr,
                      igm_pair_result* per_pair,                         /* (npairs) or NULL */
                      igm_actdist_row* rows, int64_t row_capacity,       /* CSR pair order   */
                      int64_t* nrows_out);                               /* host pointer     */

/* Next-iteration plast (ActivationDistanceStep.setup:144-160 applied to the rows
 * this A-step emitted): pairs[q].plast = float32('%.4f' % p_q) if the pair emitted
 * rows, else 0.  Valid when the same pair list is used again (same sigma). */
int igm_astep_update_plast(igm_ctx* ctx, uint32_t flags, igm_pair* pairs, int64_t npairs,
                           const igm_pair_result* per_pair);

/* ---- A-steps of configurations D/E ------------------------------------------
 * DamID: DamidActivationDistanceStep.task over ALL selected loci in one call
 * (igm/steps/DamidActivationDistanceStep.py:223-287; get_damid_actdist_I :376-471),
 * shapes 'sphere' (shape 0, nucleus_param[0] = radius) and 'ellipsoid' (shape 1,
 * nucleus_param[0..2] = semiaxes), followed by the "%6d %.5f %.5f" text round trip
 * of task()/reduce() (:35, :286, :308): rows are bit-exact
 * {i, float32(float('%.5f' % ad)), float32(float('%.5f' % p))} for every copy i of
 * every locus, in locus order.  loci[q] is a haploid locus, p_exp[q]/plast[q] the
 * float32 values setup() stores (:199-217).  per_locus[q] (nullable) reports ad, p,
 * pnow, o (-1 when p <= 0: the dist is then 2) and nrows. */
/* shape 2 = exp_map: get_damid_actdist_exp (:475-577) with snormsq_exp (:79-115) on the
 * volumetric maps staged by igm_mstep_set_volumes (struct_map = the map of every
 * structure, volumes_idx); distances ascending, pnow = count(d^2 >= contact_range),
 * dist 1e-9 when p <= 0 (nucleus_param and radii unused). */
#define IGM_DAMID_SPHERE 0
#define IGM_DAMID_ELLIPSOID 1
#define IGM_DAMID_EXP_MAP 2

typedef struct {
    int32_t loc; /* diploid bead index                               */
    float dist;  /* damid_actdist.hdf5 {loc i4, dist f4, prob f4}    */
    float prob;
} igm_damid_row;

int igm_damid_actdist(igm_ctx* ctx, uint32_t flags,
                      const float* xyz, int32_t nbead, int32_t nstruct, /* bead-major (nbead, nstruct, 3) */
                      const float* radii,
                      const int32_t* copy_ptr, const int32_t* copy_idx, int32_t nhap,
                      const int32_t* loci, const float* p_exp, const float* plast, int32_t nloci,
                      int32_t it_corr, double contact_range, int32_t shape, const double* nucleus_param,
                      igm_pair_result* per_locus,                  /* (nloci) or NULL */
                      igm_damid_row* rows, int64_t row_capacity,
                      int64_t* nrows_out);                         /* host pointer    */

/* FISH: FishAssignmentStep.task (igm/steps/FishAssignmentStep.py:188-242) for all
 * items at once.  kind 0: items = probes (haploid loci), per structure the min and
 * max over the copies of |x| (get_rad_dists, :44-58); kind 1: items = (i, j) pairs,
 * min/max over every copy pair of |x_a - x_b| (get_pair_dists' documented intent,
 * :23-41).  Distances are float32 np.linalg.norm values.  Each structure's rank
 * r = argsort(argsort(d)) (:60-77; ties in structure order) selects the target:
 * out[q, s] = target[q, r].  target_* / out_* / dist_* are (nitems, nstruct) f32;
 * every output pointer may be NULL (then its target may be NULL too). */
int igm_fish_assign(igm_ctx* ctx, uint32_t flags,
                    const float* xyz, int32_t nbead, int32_t nstruct,
                    const int32_t* copy_ptr, const int32_t* copy_idx, int32_t nhap,
                    int32_t kind, const int32_t* items, int32_t nitems,
                    const float* target_min, const float* target_max,
                    float* out_min, float* out_max, float* dist_min, float* dist_max);

/* Polymer distances: PolymerAssignmentStep.task (igm/steps/PolymerAssignmentStep.py:
 * 84-129) for all loci at once.  For locus i (0 <= i < nbead - 1) the S float32
 * distances |x_i - x_(i+1)| (get_polymer_dists, :24-32) are ranked -- argsort(argsort)
 * with ties in structure order -- and structure s receives the rank-th smallest of the
 * S values drawn by np.random.choice(edges, S, p=prob) (:113): uniforms[q, s] are the
 * random_sample() draws of that call for loci[q] (the caller's RandomState, in the
 * reference's locus order), a draw's bin is searchsorted(cumsum(p) / sum, u, 'right').
 * nn_dist (nloci, nstruct) f32 = the float64 edge value rounded to float32 (the 'f4'
 * dataset of reduce(), :158-162); dist (nloci, nstruct) f32 or NULL.  Host pointers
 * for edges / prob (nbins float64 each). */
int igm_polymer_assign(igm_ctx* ctx, uint32_t flags,
                       const float* xyz, int32_t nbead, int32_t nstruct,
                       const int32_t* loci, int32_t nloci, const double* uniforms,
                       int32_t nbins, const double* edges, const double* prob,
                       float* nn_dist, float* dist);

/* Population contact map: the simulated Hi-C counts HicEvaluationStep.reduce
 * (igm/steps/HicEvaluationStep.py:96-179) builds with HssFile.buildContactMap
 * (contactRange) at :109 (alabtools, absent here: the contact test restated is the
 * IGM Hi-C one, |x_i - x_j| (float32 norm, inter_hic.py:47) <= fl32(contact_range *
 * fl32(r_i + r_j))); the commented-out task of HicEvaluationStep.py:89-91 uses a
 * strict '<', which differs only for a distance exactly at the bound).
 * counts (nbead, nbead) int32, symmetric, diagonal included, =
 * the number of structures in contact; the caller divides by nstruct and sums the
 * copies (Contactmatrix.sumCopies, :111-112). */
int igm_contact_map(igm_ctx* ctx, uint32_t flags,
                    const float* xyz, int32_t nbead, int32_t nstruct,
                    const float* radii, double contact_range, int32_t* counts);

/* The same counts with the copies summed on the device (Contactmatrix.sumCopies,
 * HicEvaluationStep.py:111-112): counts (nhap, nhap) int32 = sum over the copy pairs
 * (a_k, b_l) of the diploid counts -- reduce()'s matrix before the division by nstruct,
 * without the (nbead, nbead) intermediate (3.6 GB at 200 kb).  copy_ptr / copy_idx
 * (host pointers, CSR of index.copy_index) must cover every bead exactly once. */
int igm_contact_map_haploid(igm_ctx* ctx, uint32_t flags,
                            const float* xyz, int32_t nbead, int32_t nstruct,
                            const float* radii, double contact_range,
                            const int32_t* copy_ptr, const int32_t* copy_idx, int32_t nhap, int32_t* counts);

/* SPRITE: SpriteAssignmentStep.task (igm/steps/SpriteAssignmentStep.py:105-160):
 * compute_gyration_radius (igm/cython_compiled/sprite.pyx:104-283, get_rg2s_cpp
 * cpp_sprite_assignment.cpp:49-143) for every (cluster, structure), then keep_best.
 * A "region" is a haploid segment with its copies alt_bead[alt_ptr[r]..alt_ptr[r+1]).
 * Cluster c has the segments seg_region[seg_ptr[c]..seg_ptr[c+1]) in output order
 * and the representatives rep_region[rep_ptr[c]..rep_ptr[c+1]) (one per chromosome,
 * drawn by the caller as sprite.pyx:231 does); seg_rep[g] is the slot of segment
 * g's chromosome among its cluster's representatives.  A cluster without
 * representatives is a single-chromosome cluster (every copy k is one group).
 * Outputs: rg2_out (ncluster, nstruct) f32 (nullable); best_idx/best_rg2
 * (ncluster, keep_best); best_sel: cluster c's (keep_best, nseg_c) selected beads at
 * offset seg_ptr[c] * keep_best.  Host pointers only (the CSR arrays are validated). */
int igm_sprite_assign(igm_ctx* ctx, uint32_t flags,
                      const float* xyz, int32_t nbead, int32_t nstruct,
                      int32_t ncluster, const int32_t* seg_ptr, const int32_t* seg_region,
                      const int32_t* seg_rep, const int32_t* rep_ptr, const int32_t* rep_region,
                      int32_t nregion, const int32_t* alt_ptr, const int32_t* alt_bead,
                      int32_t keep_best, float* rg2_out,
                      int32_t* best_idx, float* best_rg2, int32_t* best_sel);

/* DamID lamina envelope membership (M-step restraint assembly, config D):
 * Damid._apply_envelope (igm/restraints/damid.py:112-143) for every structure at once.
 * out_flags[s, a] = base_flags[a] | (env_bit if some DamID row {loc = a, dist = d}
 * has snormsq_ellipsoid(x_sa, semiaxes * (1 - contact_range), r_a) >= d^2), bit-exact
 * with the reference's NumPy 1.x arithmetic.  xyz is the M-step layout
 * (nstruct, natom, 3); the result feeds igm_mstep_run with IGM_MSTEP_STRUCT_FLAGS and
 * an envelope whose k is -contact_kspring.  n_selected (nullable): rows selected per
 * structure (the restraint's rnum). */
int igm_damid_select(igm_ctx* ctx, uint32_t flags, int32_t nstruct, int32_t natom, const float* xyz,
                     const float* radii, const igm_damid_row* rows, int64_t nrows,
                     const double* semiaxes, double contact_range, uint32_t env_bit,
                     const uint32_t* base_flags, uint32_t* out_flags, int32_t* n_selected);

/* Volumetric nuclear-body maps (VolumeFile .bin, igm/utils/files.py:137-166): header
 * int32 body_idx (0 nucleus, 1 nucleolus), int32[3] nvoxel, f32[3] center, origin, grid,
 * then int32 [nx][ny][nz][4] = (nearest-lamina voxel i, j, k, inside flag).
 * The LAMMPS fix's force form is not in the reference (lammpgen is external, SURVEY
 * M7d: parity unpinned).  Implemented form, per member atom of a volume envelope:
 *   v = round((x - envf*origin) / (envf*grid)) clamped to the grid; if the voxel
 *   violates the restraint (nucleus, k>0: outside; nucleolus, k>0: inside; k<0: the
 *   opposite, as ExpEnvelope.getScores, forces.py:306-417) the atom is pulled to the
 *   centre of its nearest lamina voxel p = envf*(origin + grid*edt(v)):
 *   E = |k|/2 |x - p|^2, F = -|k| (x - p).
 * Violation scores restate ExpEnvelope.getScores exactly (contact_range 0.95 geometry
 * shrink for k<0, its index quirks included). */
typedef struct {
    int32_t body_idx;
    int32_t nvoxel[3];
    float center[3], origin[3], grid[3];
    const int32_t* voxels; /* host pointer: nx*ny*nz*4 int32 */
} igm_volume_map;

/* Stage maps in the context for later igm_mstep_* calls: struct_map[s] selects the
 * map of structure s of a batch (volumes_idx[sid % len], ModelingStep.py:265-270);
 * NULL = map 0 for every structure.  nmap = 0 clears. */
int igm_mstep_set_volumes(igm_ctx* ctx, int32_t nmap, const igm_volume_map* maps,
                          const int32_t* struct_map, int32_t nstruct);

/* ---- M-step ---------------------------------------------------------------
 * Batched replacement of lammps.optimize (lammps.py:361-492): the protocol of
 * create_lammps_script (lammps.py:149-358) -- per stage: fix adapt of the soft
 * prefactor, envelope scaling, optional relax run, velocity create, temp/rescale
 * ramp, nve/limit -- followed by min_style cg.  One structure per workgroup:
 * structures of up to 3072 atoms (2 Mb diploid) keep positions and the Verlet
 * list in LDS; larger ones (200 kb diploid: 29 838 beads) keep them in HBM.
 */
#define IGM_MAX_STAGES 16
#define IGM_MAX_ENVELOPES 4

typedef struct {
    int32_t nstages;
    int32_t mdsteps[IGM_MAX_STAGES];
    double tstart[IGM_MAX_STAGES];
    double tstop[IGM_MAX_STAGES];
    double evfactor[IGM_MAX_STAGES];  /* fix adapt 'pair soft a' scale   */
    double envfactor[IGM_MAX_STAGES]; /* semiaxes * envf                 */
    int32_t relax_steps;              /* 0: no relax run                 */
    double relax_temperature;
    double relax_max_velocity;
    double timestep;     /* 0.25                                       */
    double max_velocity; /* nve/limit xmax (distance per step)         */
    double t_window;     /* temp/rescale window (0.1)                  */
    double t_fraction;   /* temp/rescale fraction (1.0)                */
    double etol, ftol;   /* minimize etol ftol                         */
    int32_t max_cg_iter, max_cg_eval;
    double dmax;         /* min_modify dmax (LAMMPS default 0.1)       */
    double evfactor_base;/* Steric k -> LammpsModel.evfactor           */
    double skin;         /* neighbour skin (LAMMPS: 'neighbor maxrad') */
    int32_t nenvelopes;
    double env_semiaxes[IGM_MAX_ENVELOPES][3];
    double env_k[IGM_MAX_ENVELOPES];
    int32_t neigh_capacity; /* HBM neighbour-list budget, mean entries per atom (0 = 64); atoms past
                               the budget take their pair forces from a walk of the build-time cell grid.
                               The population engine (structures too large for LDS) lists up to 256
                               entries per atom when this is 0 or 64, else min(this, 256); its
                               HBM is ~(120 + 2 x entries + 8 x max bond degree) B per atom per
                               structure (the 256-entry lists alone 15.3 GB for 1000 x 29 839 atoms), checked against the free
                               HBM before the run (IGM_E_NOMEM names the per-structure cost) */
    int32_t flags;          /* IGM_MSTEP_* below                        */
    int32_t env_kind[IGM_MAX_ENVELOPES]; /* IGM_ENV_ELLIPSOID (0) or IGM_ENV_VOLUME (1)  */
} igm_mstep_params;

/* envelope kinds (igm_mstep_params.env_kind) */
#define IGM_ENV_ELLIPSOID 0 /* fix ellipsoidalenvelope a b c k (lammps.py:292-303)              */
#define IGM_ENV_VOLUME 1    /* fix volumetricrestraint file envf k (lammps.py:305-310) with the
                               map of igm_mstep_set_volumes; env_semiaxes unused */

/* igm_mstep_params.flags */
#define IGM_MSTEP_FORCE_GLOBAL 0x1 /* use the HBM-resident kernels even when a structure fits in LDS */
#define IGM_MSTEP_STRUCT_FLAGS 0x2 /* atom_flags is (nstruct, natom): per-structure envelope membership
                                      (DamID) and active/inactive centroid slots (SPRITE); the
                                      IGM_ATOM_BEAD bit must be the same in every structure */
/* 0x4 is retired (round 3's domain-decomposed engine, 2x slower than the population engine on
   the 200 kb model, profiles/history_r01_r04.md): igm_mstep_run returns IGM_E_UNSUPPORTED for it */

/* atom flags (per atom, shared by all structures of a batch) */
#define IGM_ATOM_BEAD 0x1u   /* takes part in the soft pair potential       */
#define IGM_ATOM_FIXED 0x2u  /* setforce 0 / not integrated (static dummy)   */
#define IGM_ATOM_ENV0 0x10u  /* member of envelope e: IGM_ATOM_ENV0 << e     */

typedef struct {
    uint32_t i, j; /* atom indices; bit 31 of j set = harmonic_lower_bound */
    float r0, k;   /* E = k (r - r0)^2 beyond the bound (bond_harmonic form) */
} igm_bond;

typedef struct {
    double final_energy; /* E_pair + E_bond + sum E_env after CG ('final-energy') */
    double pair_energy;  /* thermo epair                                        */
    double bond_energy;  /* thermo ebond                                        */
    double env_energy[IGM_MAX_ENVELOPES]; /* thermo f_envelope<e>               */
    double temp;         /* thermo temp (group all)                             */
    double einitial;     /* energy at the start of CG                           */
    double fnorm_final;  /* |F|_2 at the end of CG                              */
    int32_t cg_iters, cg_evals, stop_reason, nrebuild;
} igm_opt_info;

/* Run the whole protocol for `nstruct` structures of `natom` atoms each.
 *   xyz       (nstruct, natom, 3) f32, in/out
 *   radii     (natom) f32; atom_flags (natom), or (nstruct, natom) with IGM_MSTEP_STRUCT_FLAGS
 *   bonds     shared bonds (polymer) + per-structure bonds (Hi-C ...):
 *             shared_bonds[nshared]; sbond_ptr[nstruct+1] into sbonds[]
 *   seeds     (nstruct) LAMMPS 'velocity create' seed of stage 0 (stage k: +k)
 *   info      (nstruct) or NULL                                              */
int igm_mstep_run(igm_ctx* ctx, uint32_t flags, const igm_mstep_params* prm,
                  int32_t nstruct, int32_t natom, float* xyz,
                  const float* radii, const uint32_t* atom_flags,
                  const igm_bond* shared_bonds, int64_t nshared,
                  const int64_t* sbond_ptr, const igm_bond* sbonds,
                  const int32_t* seeds, igm_opt_info* info);

/* Energy/force evaluation only (parity harness for the force field):
 * forces (nstruct, natom, 3) f32 and per-structure energies. evf/envf are the
 * stage factors to apply.  energies: (nstruct, 3 + IGM_MAX_ENVELOPES) f64 =
 * {total, pair, bond, env0..env3}.  Default: the f64 path of the CG kernel;
 * with IGM_F32_PATH: the f32 path of the MD kernel (energies are NaN). */
int igm_mstep_forces(igm_ctx* ctx, uint32_t flags, const igm_mstep_params* prm,
                     int32_t nstruct, int32_t natom, const float* xyz,
                     const float* radii, const uint32_t* atom_flags,
                     const igm_bond* shared_bonds, int64_t nshared,
                     const int64_t* sbond_ptr, const igm_bond* sbonds,
                     double evf, double envf, float* forces, double* energies);

/* Short deterministic MD segment (parity harness): `nsteps` nve/limit steps
 * with temp/rescale ramp t0->t1 from the given velocities (no velocity create).
 * v (nstruct, natom, 3) in/out. */
int igm_mstep_md(igm_ctx* ctx, uint32_t flags, const igm_mstep_params* prm,
                 int32_t nstruct, int32_t natom, float* xyz, float* v,
                 const float* radii, const uint32_t* atom_flags,
                 const igm_bond* shared_bonds, int64_t nshared,
                 const int64_t* sbond_ptr, const igm_bond* sbonds,
                 double evf, double envf, double t0, double t1, double max_velocity,
                 int32_t nsteps);

/* LAMMPS 'velocity <group> create T seed' as the reference script issues it
 * (lammps.py:322,335: dist uniform, loop all, mom yes, Park-Miller RanPark):
 * one velocity set per seed, atoms with IGM_ATOM_FIXED get 0 (not in the
 * 'nonfixed' group) but still consume their random numbers.  v: (nseed, natom, 3). */
int igm_velocity_create(igm_ctx* ctx, uint32_t flags, int32_t nseed, int32_t natom,
                        const uint32_t* atom_flags, const int32_t* seeds, double temperature,
                        float* v);

/* Profiling aid: with IGM_PROF set in the environment, the LDS-path anneal kernel
 * accumulates shader-clock cycles; out[6] = {neighbour builds, force phases, rest,
 * force evaluations, builds, list-fill walks (part of the builds)} summed over the
 * structures of the last launch. */
int igm_mstep_last_profile(igm_ctx* ctx, unsigned long long* out);

/* ---- M-step restraint assembly: Hi-C contact selection ---------------------
 * interHiC/intraHiC._apply (restraints/inter_hic.py:294-312, intra_hic.py) for
 * every actdist row and every structure: a bond (i, j) is imposed when
 * ||x_i - x_j|| <= dist (f32, no FMA) and the chromosome test holds.
 *   xyz (nstruct, natom, 3) struct-major; act rows (n_act): igm_astep_actdist output;
 *   chrom (natom); output per-structure CSR of bonds, inter rows first then
 *   intra rows (the reference order), r0 = cr*(r_i + r_j), k; out_class (may be
 *   NULL) receives inter_class / intra_class for each bond (violation classes).
 * Two-phase: call with out_bonds == NULL to get out_ptr (nstruct+1) filled and
 * the total in *ntotal; then call again with out_bonds sized *ntotal. */
int igm_hic_select(igm_ctx* ctx, uint32_t flags,
                   int32_t nstruct, int32_t natom, const float* xyz,
                   const float* radii, const int32_t* chrom,
                   const igm_actdist_row* act, /* the A-step rows (actdist.hdf5 row/col/dist/prob) */
                   int64_t n_act, double contact_range, double kspring,
                   int32_t inter_class, int32_t intra_class,
                   int64_t* out_ptr, igm_bond* out_bonds, int32_t* out_class, int64_t* ntotal);

/* Population layout change between the .hss / A-step layout (bead-major
 * (nbead, nstruct, 3), core/step.py:373) and the M-step layout (struct-major
 * (nstruct, natom, 3), natom >= nbead; extra atoms left untouched).
 * direction 0: bead-major -> struct-major; 1: struct-major -> bead-major. */
int igm_population_transpose(igm_ctx* ctx, uint32_t flags, int32_t nbead, int32_t nstruct, int32_t natom,
                             const float* src, float* dst, int32_t direction);

/* ---- M-step violation scoring (ModelingStep.py:511-557,859-869) ------------
 * For each structure and each restraint class c -- bond classes 0..nclass_bonds-1
 * (class ids parallel to shared_bonds / sbonds), then envelope e as class
 * nclass_bonds + e -- the ModelingStep.task record: histogram of 100 bins on
 * [0,1] + overflow (np.histogram semantics), violated_restr (ratio != 0),
 * n_violations (ratio > tol) and n_imposed.
 *   bond ratio    k (r - d) / (k d) past the bound, d = class_cr[c] * f32(r_i + r_j)
 *                 in f64 (forces.py:131-139,178-186); class_cr[c] <= 0: d = bond r0
 *   envelope      EllipticEnvelope.getScores (forces.py:222-247) with the base
 *                 semiaxes, scale env_scale[e] (0.1 * mean(abc), envelope.py:51)
 * stats: (nstruct, nclass_bonds + nenvelopes, 104) int64 =
 *        {counts[101], violated_restr, n_violations, n_imposed}. */
int igm_mstep_violations(igm_ctx* ctx, uint32_t flags, const igm_mstep_params* prm,
                         int32_t nstruct, int32_t natom, const float* xyz,
                         const float* radii, const uint32_t* atom_flags,
                         const igm_bond* shared_bonds, const int32_t* shared_class, int64_t nshared,
                         const int64_t* sbond_ptr, const igm_bond* sbonds, const int32_t* sclass,
                         int32_t nclass_bonds, const double* class_cr, const double* env_scale, double tol,
                         int64_t* stats);

#ifdef __cplusplus
}
#endif
#endif /* IGM_HIP_H */
