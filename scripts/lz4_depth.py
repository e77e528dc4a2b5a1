import sys, numpy as np
sys.path.insert(0, '/root/repo')
import bench
from redpanda_amd import abi, engine
cfg = bench.CONFIGS['c3']
spec = engine.make_spec(seed=0x5EED0003, partitions=cfg['partitions'], **cfg['spec'])
spec.ops = abi.OPS_PRODUCE | abi.OP_DECOMP; spec.payload = abi.PAYLOAD_TEXT
data, descs = engine.build_arena(spec, 8)
for i in range(4):
    off, ln = int(descs['offset'][i]), int(descs['length'][i])
    body = bytes(data[off+61:off+ln])
    # LZ4 frame: magic 4, FLG, BD, [content size 8], HC
    flg = body[4]; hl = 7 + (8 if flg & 8 else 0) + (4 if flg & 1 else 0)
    bh = int.from_bytes(body[hl:hl+4], 'little'); sz = bh & 0x7fffffff
    blk = body[hl+4:hl+4+sz]
    ip = op = 0; seqs = []
    while ip < len(blk):
        tok = blk[ip]; ip += 1; ll = tok >> 4
        if ll == 15:
            while True:
                s = blk[ip]; ip += 1; ll += s
                if s != 255: break
        lit = (op, ll); ip += ll; op += ll
        if ip >= len(blk): break
        o = blk[ip] | blk[ip+1] << 8; ip += 2; ml = tok & 15
        if ml == 15:
            while True:
                s = blk[ip]; ip += 1; ml += s
                if s != 255: break
        ml += 4
        seqs.append((op, o, ml)); op += ml
    # level per output byte
    lev = np.zeros(op + 1, dtype=np.int32)
    D = 0
    for (m, o, ml) in seqs:
        a = m - o; n = min(o, ml)
        l = 1 + int(lev[a:a+n].max()) if n > 0 else 1
        lev[m:m+ml] = l; D = max(D, l)
    offs = np.array([o for _, o, _ in seqs])
    print(f"block {i}: in {len(blk)} out {op} tokens {len(seqs)} depth {D} median off {int(np.median(offs))} >4K {np.mean(offs>4096):.2f} mean ml {np.mean([s[2] for s in seqs]):.1f}")
