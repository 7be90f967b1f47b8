# LDS bank-conflict simulator for the NTN P-image accesses (MI355X_MICROARCH.md LDS table)
import itertools, random
def cyc_read(addrs, groups, width):   # reads: 64 banks, bank=(a/4)%64; returns conflict cycles (extra)
    extra=0
    for g in groups:
        banks={}
        for l in g:
            a=addrs[l]
            if a is None: continue
            for w in range(width//4):
                b=((a//4)+w)%64
                banks.setdefault(b,set()).add((a//4)+w)
        m=max((len(v) for v in banks.values()), default=1)
        extra+=m-1
    return extra
def cyc_write(addrs, groups, width):   # writes: 32 banks
    extra=0
    for g in groups:
        banks={}
        for l in g:
            a=addrs[l]
            if a is None: continue
            for w in range(width//4):
                b=((a//4)+w)%32
                banks.setdefault(b,set()).add((a//4)+w)
        m=max((len(v) for v in banks.values()), default=1)
        extra+=m-1
    return extra
G32=[list(range(32)),list(range(32,64))]
G16=[list(range(i,i+16)) for i in range(0,64,16)]
GB128=[[0,1,2,3,12,13,14,15]+list(range(20,28)),list(range(4,12))+[16,17,18,19,28,29,30,31]]
GB128=GB128+[[x+32 for x in g] for g in GB128]
def evaluate(X, IMG1=2048, N=5, G=2, SG=3):
    # X: list of 16 chunk-XORs (8-B chunks, 0..15)
    tot={}
    def addr(img,row,chunk): return img*IMG1 + row*128 + ((chunk ^ X[row])<<3)
    # R1 p_rows: lane -> row n, 16B at chunk pair 8kb+2q
    r1=0
    for kb in range(2):
        A=[addr(0,l&15,8*kb+2*(l>>4)) for l in range(64)]
        r1+=cyc_read(A,GB128,16)
    tot['R1']=r1
    # R2 Pt tr: rows 4q+(n>>2), chunk 4mb+(n&3)
    r2=0
    for mb in range(3):
        A=[addr(0,4*(l>>4)+((l&15)>>2),4*mb+(l&3)) for l in range(64)]
        r2+=cyc_read(A,G32,8)
    tot['R2']=r2
    # W2 D write: row n, chunk 4mb+q
    w2=0
    for mb in range(3):
        A=[addr(0,l&15,4*mb+(l>>4)) for l in range(64)]
        w2+=cyc_write(A,G16,8)
    tot['W2']=w2
    # W1 P write: lane n<G*N -> image n//N, row sl*N + n%N, chunk 4mb+q
    w1=0
    for sl in range(SG):
        for mb in range(3):
            A=[addr((l&15)//N, sl*N+(l&15)%N, 4*mb+(l>>4)) if (l&15)<G*N else None for l in range(64)]
            w1+=cyc_write(A,G16,8)
    tot['W1']=w1
    # R3 Bd: lane n<G*N -> image n//N row sl*N+n%N, 16B chunk pair 8kb+2q; others zero block (broadcast; ignore)
    r3=0
    for sl in range(SG):
        for kb in range(2):
            A=[addr((l&15)//N, sl*N+(l&15)%N, 8*kb+2*(l>>4)) if (l&15)<G*N else None for l in range(64)]
            r3+=cyc_read(A,GB128,16)
    tot['R3']=r3
    return tot
cur=[((r&6)<<1) for r in range(16)]
print("current", evaluate(cur))
