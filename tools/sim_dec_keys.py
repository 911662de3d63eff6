# Diagnostic (not product): LDS bank model of tdt_decode.h decode_fast key writes on C3 blobs,
# with and without an XOR swizzle of the head-key address.
# LDS bank-conflict model of decode_fast's key writes (ds_write_b16, 2 x 32-lane groups, 32
# banks of 4 B): per instruction j (pair j of each lane's 8) the extra cycles over 1 per group.
import numpy as np, sys
sys.path.insert(0,'/root/repo')
from oracle.oracle import Oracle
rng=np.random.default_rng(1)
orc=Oracle()
def blob_pairs(n=65536):
    x=rng.normal(0,0.01,n//4).astype(np.float32); x[rng.random(x.size)<0.7]=0
    b=np.frombuffer(orc.encode(x.view(np.uint8),bandwidth=10.0),np.uint8)
    ns=int.from_bytes(b[8:12],'little'); ws=int.from_bytes(b[12:16],'little')
    mp=[int.from_bytes(b[20+4*i:24+4*i],'little') for i in range(ws)]
    off=20+4*ws; streams=[]
    for s in range(ns):
        L=int.from_bytes(b[off:off+4],'little'); off+=4
        streams.append(b[off:off+L]); off+=L
    return mp,streams
def sim(swz, trials=20):
    tot=0; base=0; writes=0
    for t in range(trials):
        mp,streams=blob_pairs()
        # r=0: stream of mapping[0]; seg: 4*k
        m0=mp[0]; segs={s:4*mp.count(s) for s in set(mp)}
        order=[m0]+[s for s in sorted(set(mp)) if s!=m0]
        hb=0
        for r,s in enumerate(order):
            st=streams[s]; cnt=st[0::2].astype(np.int64)
            start=np.concatenate([[0],np.cumsum(cnt)[:-1]])
            seg=segs[s]; wlen=3*64*seg
            hbase = 0 if r==0 else 2*(3*64*segs[order[0]]+16)
            if swz: start=start ^ (((start>>6)&7)<<3)
            np_=len(cnt)
            for b0 in range(0,np_,512):
                blk=start[b0:b0+512]
                if len(blk)<512: blk=np.concatenate([blk,np.full(512-len(blk),-1)])
                blk=blk.reshape(64,8)
                lo=blk[blk>=0].min(); hi=blk.max()
                for w0 in range((lo//wlen)*wlen, hi+1, wlen):
                    rel=blk-w0
                    slot=np.where((rel>=0)&(rel<wlen),rel,wlen)
                    addr=hbase+2*slot
                    for j in range(8):
                        a=addr[:,j]
                        for g in (a[:32],a[32:]):
                            dw=np.unique(g//4)
                            banks=dw%32
                            c=np.bincount(banks,minlength=32).max()
                            tot+=c; base+=1
                        writes+=1
    return tot/base, writes
for swz in (0,1):
    print('swizzle',swz,'avg cycles per 32-lane group', sim(swz,5))
