/* igm_io.h -- native .hss / actdist.hdf5 I/O for the IGM population.
 *
 * A self-contained reader and writer for the subset of HDF5 that IGM's files use,
 * so the population, the A-step rows and the summary move between steps without
 * h5py/libhdf5 (neither is importable by this package's Python):
 *
 *   .hss (alabtools HssFile, written through h5py, read by core/step.py:346-396,
 *        ModelingStep.py:578-783, _preprocess.py:90-188):
 *        attrs nbead, nstruct (int64), version (int32), violation (float64);
 *        datasets coordinates (nbead, nstruct, 3) f4, radii f4, index/{chrom, copy,
 *        start, end, chrom_sizes i4, chromstr, label S10, copy_index, custom_tracks
 *        vlen str}, genome/{assembly vlen str, chroms S10, lengths, origins i4},
 *        envelope/{shape vlen str, volume f8, params}, summary / config_data vlen str.
 *   actdist.hdf5 (ActivationDistanceStep.py:285-289): row, col i4, dist, prob f4.
 *
 * Reader: superblock 0/1, symbol-table groups (B-tree v1 + local heap), version-1
 * object headers with continuation blocks, dataspace v1/v2, fixed-point / float /
 * fixed string / variable-length string types, layouts compact / contiguous /
 * chunked (B-tree v1 chunk index, deflate + shuffle + fletcher32 filters), attributes
 * v1-v3, global-heap vlen data.  Anything else fails with a message.
 * Writer: superblock 0, symbol-table groups, version-1 object headers, contiguous
 * unfiltered datasets, scalar or simple dataspaces, vlen strings in one global heap
 * collection -- the layout h5py produces with its default (earliest) file format,
 * except that datasets are contiguous rather than chunked.
 *
 * All functions return 0 on success and a negative code on failure; the message is
 * igm_io_last_error().  Numeric data is little-endian, row-major.
 */
#ifndef IGM_IO_H
#define IGM_IO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* datatype classes (HDF5 class numbers) */
#define IGM_H5_INT 0     /* fixed-point, 1/2/4/8 bytes, signed or unsigned */
#define IGM_H5_FLOAT 1   /* IEEE 4 or 8 bytes */
#define IGM_H5_STRING 3  /* fixed-length byte string (numpy 'S<n>') */
#define IGM_H5_VLSTR 9   /* variable-length string (h5py str) */

#define IGM_H5_MAXRANK 8

typedef struct igm_h5 igm_h5;    /* an open file (read) */
typedef struct igm_h5w igm_h5w;  /* a file being written */

typedef struct {
    int32_t cls;        /* IGM_H5_* */
    int32_t size;       /* bytes per element (vlen: 16, the on-disk reference) */
    int32_t is_signed;  /* fixed-point only */
    int32_t rank;       /* 0: scalar */
    int64_t dims[IGM_H5_MAXRANK];
    int64_t nelem;
    int32_t layout;     /* 0 compact, 1 contiguous, 2 chunked, -1 attribute */
    int32_t nfilter;
    int64_t data_offset; /* contiguous: file offset of the raw data (-1 otherwise / unallocated) */
} igm_h5_info;

const char* igm_io_last_error(void);

/* ---- reading (h5py.File(path, 'r') / HssFile / h5py's dataset and attrs API) */
int igm_h5_open(const char* path, igm_h5** out);
int igm_h5_close(igm_h5* f);
/* names of the members of a group, '\n'-separated, groups with a trailing '/';
 * *needed = bytes required including the terminating 0 */
int igm_h5_list(igm_h5* f, const char* group, char* names, size_t cap, size_t* needed);
/* the attribute names of an object, '\n'-separated */
int igm_h5_attr_names(igm_h5* f, const char* path, char* names, size_t cap, size_t* needed);
/* dataset (attr == NULL) or attribute `attr` of object `path` */
int igm_h5_info_of(igm_h5* f, const char* path, const char* attr, igm_h5_info* info);
/* all elements, raw (nbytes must equal nelem * size; not for IGM_H5_VLSTR) */
int igm_h5_read(igm_h5* f, const char* path, const char* attr, void* out, size_t nbytes);
/* element `index` of a vlen string dataset/attribute: *len = its length; copies
 * min(len, cap) bytes */
int igm_h5_read_vlstr(igm_h5* f, const char* path, const char* attr, int64_t index, char* out, size_t cap,
                      size_t* len);

/* ---- writing (h5py.File(path, 'w'), create_group, create_dataset, attrs.create) */
int igm_h5w_create(const char* path, igm_h5w** out);
/* creates the group and its missing parents */
int igm_h5w_group(igm_h5w* w, const char* path);
/* a dataset (parents created); data holds nelem * size bytes, copied */
int igm_h5w_dataset(igm_h5w* w, const char* path, int32_t cls, int32_t size, int32_t is_signed, int32_t rank,
                    const int64_t* dims, const void* data);
/* a scalar vlen string dataset (attr == NULL) or attribute of `path` */
int igm_h5w_vlstr(igm_h5w* w, const char* path, const char* attr, const char* str, size_t len);
/* an attribute of the object at `path` ("/" = root) */
int igm_h5w_attr(igm_h5w* w, const char* path, const char* name, int32_t cls, int32_t size, int32_t is_signed,
                 int32_t rank, const int64_t* dims, const void* data);
/* lays the file out and writes it (atomically: path.part then rename); frees w */
int igm_h5w_close(igm_h5w* w);
/* frees w without writing */
int igm_h5w_abort(igm_h5w* w);

#ifdef __cplusplus
}
#endif
#endif
