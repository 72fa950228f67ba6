"""Volumetric nuclear-body maps (configuration E): the VolumeFile `.bin` format
(igm/utils/files.py:137-166) and their staging for the M-step.

  read_volume / write_volume  -- header int32 body_idx, int32[3] nvoxel, f32[3] center,
                                 origin, grid, then int32 [nx][ny][nz][4] = (nearest
                                 lamina voxel i, j, k, inside flag), native byte order
  sphere_map                  -- a voxelized sphere with its EDT nearest-lamina indices
                                 (100 nm grid)
  stage                       -- igm_mstep_set_volumes: the maps and the per-structure
                                 map index volumes_idx[sid % len] (ModelingStep.py:265-270)
"""
import ctypes
import struct

import numpy as np

from . import _lib


def read_volume(path):
    with open(path, 'rb') as g:
        body_idx = struct.unpack('i', g.read(4))[0]
        nvoxel = struct.unpack('iii', g.read(12))
        center = struct.unpack('fff', g.read(12))
        origin = struct.unpack('fff', g.read(12))
        grid = struct.unpack('fff', g.read(12))
        n = nvoxel[0] * nvoxel[1] * nvoxel[2] * 4
        mat = np.frombuffer(g.read(4 * n), dtype=np.int32).reshape(nvoxel[0], nvoxel[1], nvoxel[2], 4)
    return dict(body_idx=body_idx, nvoxel=np.array(nvoxel, np.int32), center=np.array(center, np.float32),
                origin=np.array(origin, np.float32), grid=np.array(grid, np.float32), matrice=mat.copy())


def write_volume(path, vol):
    with open(path, 'wb') as g:
        g.write(struct.pack('i', int(vol['body_idx'])))
        g.write(struct.pack('iii', *[int(v) for v in vol['nvoxel']]))
        for key in ('center', 'origin', 'grid'):
            g.write(struct.pack('fff', *[float(v) for v in vol[key]]))
        g.write(np.ascontiguousarray(vol['matrice'], np.int32).tobytes())


def sphere_map(radius=5500.0, grid=100.0, margin=3, body_idx=0, center=(0.0, 0.0, 0.0)):
    """A voxelized sphere: voxel v is inside when its centre lies within `radius`;
    lamina voxels are inside voxels with an outside 6-neighbour; every voxel carries
    the index of its nearest lamina voxel (Euclidean distance transform)."""
    from scipy import ndimage
    n = int(np.ceil(2 * radius / grid)) + 2 * margin + 1
    origin = np.asarray(center, np.float64) - grid * (n - 1) / 2.0
    ax = [origin[d] + grid * np.arange(n) for d in range(3)]
    X, Y, Z = np.meshgrid(ax[0] - center[0], ax[1] - center[1], ax[2] - center[2], indexing='ij')
    inside = (X * X + Y * Y + Z * Z) <= radius * radius
    er = ndimage.binary_erosion(inside, structure=ndimage.generate_binary_structure(3, 1), border_value=0)
    lamina = inside & ~er
    _, idx = ndimage.distance_transform_edt(~lamina, return_indices=True)
    mat = np.zeros((n, n, n, 4), np.int32)
    mat[..., 0], mat[..., 1], mat[..., 2] = idx[0], idx[1], idx[2]
    mat[..., 3] = inside.astype(np.int32)
    return dict(body_idx=int(body_idx), nvoxel=np.array([n, n, n], np.int32),
                center=np.asarray(center, np.float32), origin=origin.astype(np.float32),
                grid=np.array([grid] * 3, np.float32), matrice=mat)


def stage(ctx, vols, struct_map=None):
    """igm_mstep_set_volumes(maps, struct_map); the arrays stay referenced by ctx."""
    arr = (_lib.VolumeMap * max(len(vols), 1))()
    keep = []
    for m, v in enumerate(vols):
        mat = np.ascontiguousarray(v['matrice'], np.int32)
        keep.append(mat)
        arr[m].body_idx = int(v['body_idx'])
        for d in range(3):
            arr[m].nvoxel[d] = int(v['nvoxel'][d])
            arr[m].center[d] = float(v['center'][d])
            arr[m].origin[d] = float(v['origin'][d])
            arr[m].grid[d] = float(v['grid'][d])
        arr[m].voxels = mat.ctypes.data
    smap = None if struct_map is None else np.ascontiguousarray(struct_map, np.int32)
    rc = ctx.lib.igm_mstep_set_volumes(ctx.h, len(vols), ctypes.addressof(arr) if vols else None,
                                       smap.ctypes.data if smap is not None else None,
                                       0 if smap is None else len(smap))
    ctx.check(rc, 'igm_mstep_set_volumes')
    ctx._volumes = (arr, keep, smap)
