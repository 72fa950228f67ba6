"""IGM's population files on the native HDF5 reader/writer (igm_amd.h5), SURVEY 8(f)2.

  .hss  alabtools HssFile, the population between steps (igm/_preprocess.py:90-188
        allocates it, core/step.py:346-396 and ModelingStep.py:578-783 read and fill
        it): attrs nbead, nstruct (int64), version (int32), violation (float64);
        coordinates (nbead, nstruct, 3) float32 BEAD-major; radii f4; index/{chrom,
        copy, start, end, chrom_sizes i4, chromstr, label S10, copy_index and
        custom_tracks JSON str}; genome/{assembly str, chroms S10, lengths, origins
        i4}; envelope/{shape str, volume f8, params}; summary / config_data JSON str.
  .hcs  alabtools Contactmatrix, the Hi-C input (ActivationDistanceStep.py:124-191):
        matrix/{indptr, indices i4, data, diagonal f4} (upper triangle, CSR) + index.
  actdist.hdf5  the A-step rows (ActivationDistanceStep.py:285-289): row, col i4,
        dist, prob f4.

Files written here keep the reference's dataset names, types and shapes; the datasets
are contiguous (not gzip-chunked), so the coordinates can be memory-mapped and updated
in place (`coordinates_memmap`) -- the M-step's reduce writes the population without
per-structure files or an h5repack pass (ModelingStep.py:578-610, 783).
"""
import json
import os

import numpy as np

from . import h5
from ._lib import row_dtype


def copy_index_json(copy_ptr, copy_idx):
    """index.copy_index as alabtools stores it: {haploid id: [diploid beads]}"""
    return json.dumps({str(h): [int(b) for b in copy_idx[copy_ptr[h]:copy_ptr[h + 1]]]
                       for h in range(len(copy_ptr) - 1)})


def copy_index_arrays(text):
    """(copy_ptr, copy_idx) of an index.copy_index JSON string (haploid order)"""
    d = json.loads(text)
    keys = sorted(d, key=int)
    ptr = np.zeros(len(keys) + 1, np.int32)
    ptr[1:] = np.cumsum([len(d[k]) for k in keys])
    idx = np.array([b for k in keys for b in d[k]], np.int32)
    return ptr, idx


def _s10(a, n):
    if a is None:
        return np.zeros(n, 'S10')
    return np.asarray(a).astype('S10')


def index_tree(chrom, copy, copy_ptr, copy_idx, chrom_sizes=None, start=None, end=None, chromstr=None,
               label=None, custom_tracks='{}'):
    n = len(chrom)
    chrom = np.asarray(chrom, np.int32)
    if chrom_sizes is None:  # alabtools Index.chrom_sizes: beads of every (chromosome, copy) run, in order
        key = chrom.astype(np.int64) * 64 + np.asarray(copy, np.int64)
        starts = np.concatenate([[0], np.nonzero(np.diff(key))[0] + 1, [n]]) if n else np.zeros(1, np.int64)
        chrom_sizes = np.diff(starts)
    return {'chrom': chrom, 'copy': np.asarray(copy, np.int32),
            'start': np.zeros(n, np.int32) if start is None else np.asarray(start, np.int32),
            'end': np.zeros(n, np.int32) if end is None else np.asarray(end, np.int32),
            'chrom_sizes': np.asarray(chrom_sizes, np.int32),
            'chromstr': _s10(chromstr, n), 'label': _s10(label if label is not None else [b'-'] * n, n),
            'copy_index': copy_index_json(copy_ptr, copy_idx), 'custom_tracks': custom_tracks}


def write_hss(path, coordinates, radii, index, genome=None, envelope=None, summary=None, config_data=None,
              violation=float('nan'), version=2):
    """A new .hss (HssFile layout).  coordinates: (nbead, nstruct, 3) bead-major;
    index: the dict of index_tree(); genome/envelope: dicts of their datasets."""
    crd = np.ascontiguousarray(coordinates, np.float32)
    nbead, nstruct = crd.shape[0], crd.shape[1]
    tree = {'@version': np.int32(version), '@violation': np.float64(violation), '@nstruct': np.int64(nstruct),
            '@nbead': np.int64(nbead), 'coordinates': crd, 'radii': np.asarray(radii, np.float32), 'index': index}
    if genome is not None:
        tree['genome'] = genome
    if envelope is not None:
        tree['envelope'] = envelope
    if summary is not None:
        tree['summary'] = summary
    if config_data is not None:
        tree['config_data'] = config_data
    h5.write(path, tree)


def read_tree(f, group='/', skip=()):
    """every dataset and attribute under `group` as a nested dict (the write() form)"""
    t = {}
    for k in f.keys(group):
        p = group.rstrip('/') + '/' + k.rstrip('/')
        if p.lstrip('/') in skip:
            continue
        t[k.rstrip('/')] = read_tree(f, p, skip) if k.endswith('/') else f.read(p)
    for k, v in f.attrs(group).items():
        t['@' + k] = v
    return t


def update_hss(path, **changes):
    """Rewrite a .hss with some members replaced (summary=..., violation=..., any
    top-level dataset): the reference's HssFile.set_* calls.  The result is
    contiguous, so a chunked (h5py-written) file becomes memory-mappable."""
    with h5.File(path) as f:
        # contiguous coordinates stream from a memory map of the old file instead of
        # being read into memory and copied (the 200 kb pop=1000 population is 360 MB)
        big = 'coordinates' not in changes and 'coordinates' in f.keys('/') and \
            f.data_offset('coordinates') is not None
        tree = read_tree(f, skip=('coordinates',) if big else ())
        if big:
            off, shape = f.data_offset('coordinates'), f.shape('coordinates')
    if big:
        tree['coordinates'] = np.memmap(path, np.float32, 'r', offset=off, shape=shape)
    for k, v in changes.items():
        if k in ('violation', 'nstruct', 'nbead', 'version'):
            tree['@' + k] = {'violation': np.float64, 'nstruct': np.int64, 'nbead': np.int64,
                             'version': np.int32}[k](v)
        else:
            tree[k] = v
    tmp = path + '.update.tmp'  # the old file is still mapped: write beside it, then rename
    h5.write(tmp, tree)
    del tree
    os.replace(tmp, path)


def coordinates_memmap(path, mode='r'):
    """the coordinates dataset (nbead, nstruct, 3) f4 as an np.memmap of the file
    (mode 'r' or 'r+'); a chunked file is rewritten contiguous first for 'r+'"""
    with h5.File(path) as f:
        off, shape = f.data_offset('coordinates'), f.shape('coordinates')
        inf = f.info('coordinates')
    if inf.cls != h5.FLOAT or inf.size != 4:
        raise OSError('%s: coordinates are not float32' % path)
    if off is None:
        if mode == 'r':
            with h5.File(path) as f:
                return f.read('coordinates')
        update_hss(path)
        return coordinates_memmap(path, mode)
    return np.memmap(path, np.float32, mode, offset=off, shape=shape)


class Hss(object):
    """HssFile's read side: nstruct, nbead, radii, index arrays, coordinates."""

    def __init__(self, path):
        self.path = path
        with h5.File(path) as f:
            a = f.attrs('/')
            self.nstruct, self.nbead = int(a['nstruct']), int(a['nbead'])
            self.version = int(a.get('version', 2))
            self.violation = float(a.get('violation', np.nan))
            self.radii = f.read('radii').astype(np.float32)
            self.chrom = f.read('index/chrom').astype(np.int32)
            self.copy = f.read('index/copy').astype(np.int32)
            self.copy_ptr, self.copy_idx = copy_index_arrays(f.read('index/copy_index'))
            self.chrom_sizes = f.read('index/chrom_sizes').astype(np.int64) if 'chrom_sizes' in f.keys('index') \
                else None
            names = f.keys('/')
            self.summary = f.read('summary') if 'summary' in names else None

    def coordinates(self, mode='r'):
        return coordinates_memmap(self.path, mode)

    def get_struct_crd(self, sid):
        return np.array(self.coordinates()[:, sid, :])


def read_hcs(path):
    """the .hcs Contactmatrix arrays ActivationDistanceStep.setup reads: CSR of the
    upper triangle (indptr, indices, data) and the haploid index chrom"""
    with h5.File(path) as f:
        return {'indptr': f.read('matrix/indptr').astype(np.int64), 'indices': f.read('matrix/indices').astype(np.int32),
                'data': f.read('matrix/data').astype(np.float32), 'chrom': f.read('index/chrom').astype(np.int32),
                'nbin': int(f.attrs('/').get('nbin', len(f.read('index/chrom'))))}


def write_actdist(path, rows):
    """actdist.hdf5 with the four datasets of ActivationDistanceStep.reduce (:285-289)"""
    tmp = path + '.tmp'
    h5.write(tmp, {'row': np.ascontiguousarray(rows['row'], np.int32),
                   'col': np.ascontiguousarray(rows['col'], np.int32),
                   'dist': np.ascontiguousarray(rows['dist'], np.float32),
                   'prob': np.ascontiguousarray(rows['prob'], np.float32)})
    os.replace(tmp, path)


def read_actdist(path):
    with h5.File(path) as f:
        cols = {k: f.read(k) for k in ('row', 'col', 'dist', 'prob')}
    rows = np.zeros(len(cols['row']), row_dtype)
    for k, v in cols.items():
        rows[k] = v
    return rows
