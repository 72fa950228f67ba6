"""An independent pure-Python walker of the HDF5 structures igm_amd's writer emits
(test infrastructure: a second reading of csrc/h5io.cpp's output that shares no code
with it).  It checks the layout rules libhdf5 relies on -- superblock 0 with the EOF
address equal to the file size, group B-trees whose SNOD entries are sorted by name
with keys equal to the last name of each node, local heaps starting with "" and
terminated by the free-list sentinel 1, version-1 object headers whose messages are
8-byte sized and fill the chunk exactly, 8-byte aligned structures, global heap
collections of >= 4096 bytes -- and returns {path: {'messages': [...], 'attrs': [...]}}."""
import struct


class Bad(AssertionError):
    pass


def _u(buf, fmt, o):
    return struct.unpack_from('<' + fmt, buf, o)


def inspect(path):
    buf = open(path, 'rb').read()
    if buf[:8] != b'\x89HDF\r\n\x1a\n':
        raise Bad('signature')
    if buf[8] != 0 or buf[13] != 8 or buf[14] != 8:
        raise Bad('superblock version / sizes')
    leafk, intk = _u(buf, 'HH', 16)
    base, fs, eof, drv = _u(buf, 'QQQQ', 24)
    if base != 0 or eof != len(buf):
        raise Bad('base %d / EOF %d vs %d bytes' % (base, eof, len(buf)))
    _, root, ctype = _u(buf, 'QQI', 56)
    out = {}

    def heap(addr):
        if buf[addr:addr + 4] != b'HEAP' or addr % 8:
            raise Bad('heap at %d' % addr)
        size, free, data = _u(buf, 'QQQ', addr + 8)
        if free != 1 or buf[data:data + 8] != b'\0' * 8 or data + size > len(buf):
            raise Bad('heap fields at %d' % addr)
        return data, size

    def name(h, off):
        d, s = h
        if off >= s:
            raise Bad('name offset')
        e = buf.index(b'\0', d + off)
        return buf[d + off:e].decode()

    def header(addr):
        if addr % 8 or buf[addr] != 1:
            raise Bad('object header at %d' % addr)
        nmsg, refc, csize = _u(buf, 'HII', addr + 2)
        if refc != 1:
            raise Bad('refcount')
        p, end, msgs = addr + 16, addr + 16 + csize, []
        while p < end:
            t, s, fl = _u(buf, 'HHB', p)
            if s % 8:
                raise Bad('message size %d not a multiple of 8' % s)
            msgs.append((t, fl, buf[p + 8:p + 8 + s]))
            p += 8 + s
        if p != end or len(msgs) != nmsg:
            raise Bad('messages do not fill the header chunk at %d' % addr)
        return msgs

    def group(addr, gpath):
        msgs = header(addr)
        st = [m for m in msgs if m[0] == 0x11]
        if len(st) != 1:
            raise Bad('group without one symbol table')
        bt, hp = struct.unpack_from('<QQ', st[0][2])
        h = heap(hp)
        if buf[bt:bt + 4] != b'TREE' or buf[bt + 4] != 0 or buf[bt + 5] != 0:
            raise Bad('group B-tree at %d' % bt)
        n = _u(buf, 'H', bt + 6)[0]
        if n > 2 * intk:
            raise Bad('B-tree overfull')
        keys = [_u(buf, 'Q', bt + 24 + 16 * i)[0] for i in range(n + 1)]
        kids = [_u(buf, 'Q', bt + 32 + 16 * i)[0] for i in range(n)]
        if keys[0] != 0:
            raise Bad('B-tree key 0')
        names = []
        for i, ch in enumerate(kids):
            if buf[ch:ch + 4] != b'SNOD' or ch % 8:
                raise Bad('SNOD at %d' % ch)
            ns = _u(buf, 'H', ch + 6)[0]
            if not 0 < ns <= 2 * leafk:
                raise Bad('SNOD size %d' % ns)
            ents = []
            for k in range(ns):
                lo, oh, ct = _u(buf, 'QQI', ch + 8 + 40 * k)
                ents.append((name(h, lo), oh, ct, _u(buf, "QQ", ch + 32 + 40 * k)))
            if name(h, keys[i + 1]) != ents[-1][0]:
                raise Bad('B-tree key %d is not the last name of its node' % (i + 1))
            names += [e[0] for e in ents]
            for nm, oh, ct, scratch in ents:
                p = gpath.rstrip('/') + '/' + nm
                if ct == 1:
                    g = group(oh, p)
                    if scratch != g:
                        raise Bad('scratch pad of %s' % p)
                else:
                    out[p] = {'messages': header(oh), 'kind': 'dataset'}
        if names != sorted(names, key=lambda x: x.encode()):
            raise Bad('group %s not sorted by name' % gpath)
        out[gpath] = {'messages': msgs, 'kind': 'group'}
        return bt, hp

    group(root, '/')
    g = buf.find(b'GCOL')
    while g >= 0:
        if g % 8 == 0 and buf[g + 4] == 1:
            if _u(buf, 'Q', g + 8)[0] < 4096:
                raise Bad('global heap collection smaller than 4096 bytes')
        g = buf.find(b'GCOL', g + 4)
    return out
