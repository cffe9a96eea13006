"""Numpy emulation of describe.hip's matrix-core blur (ORBGPU_DESC_MFMA): the
row pass as an i8 16x16x64 product (bytes as p - 128, accumulator 128 x 257),
the column pass as an f16 16x16x32 product of the row sums' low / high bytes
entering as f16 subnormals against taps x 4 / x 1024, 64 x the f32 result
rounded half to even -- against the two-pass integer blur, on random patches
(rows 43..47 and columns 48..63 filled with garbage, as the kernel reads them).
Fragment maps as the kernel builds them (c_blur_mfma); the MFMA k-order only has
to agree between A and B, which this assumes and the GPU parity tests check."""
import numpy as np
rng=np.random.default_rng(1)
tap=[18,34,49,55,49,34,18]
def f16bits(v):
    return np.float16(v).view(np.uint16)
# tables
row=np.zeros((3,64,16),np.int64); col=np.zeros((2,64,8),np.float64)
for l in range(64):
    g,c=l>>4,l&15
    for nt in range(3):
        for j in range(16):
            d=16*g+j-(16*nt+c)-1
            if 0<=d<=6: row[nt,l,j]=tap[d]
    for dd in range(2):
        for j in range(8):
            d=16*dd+4*g+(j&3)-c
            if 0<=d<=6: col[dd,l,j]=float(np.float16(tap[d]*(1024 if j>>2 else 4)))
for trial in range(200):
    P=rng.integers(0,256,(48,64)).astype(np.int64)  # rows 43.. and cols 48.. garbage
    if trial%3==0: P[:43,:48]=255
    # reference blur (exact): row sums over raw cols x+1..x+7, col over rows y..y+6
    R=np.zeros((43,40),np.int64)
    for x in range(40):
        R[:,x]=sum(tap[k]*P[:43,x+1+k] for k in range(7))
    V=np.zeros((37,40),np.int64)
    for y in range(37):
        V[y]=sum(tap[k]*R[y+k] for k in range(7))
    ref=np.clip(np.round(V/65536.0),0,255)  # numpy round = half-even
    # emulation
    out=np.zeros((48,48))
    for mx in range(3):
        D={}
        for s in range(3):
            # A[i][k] = P[16s+i][k]-128 (lane i+16*(k//16), elem k%16); B[k][j]=row[mx][lane j+16*(k//16)][k%16]
            A=P[16*s:16*s+16,:64]-128
            B=np.zeros((64,16),np.int64)
            for k in range(64):
                for j in range(16): B[k,j]=row[mx,j+16*(k//16),k%16]
            D[s]=A@B+32896   # D[i][j]: R rows 16s+i, cols 16mx+j
        for ny in range(3):
            acc=np.zeros((16,16))
            for s,dd in ((ny,0),(ny+1,1)):
                if s>2: continue
                # A2[i][k]: i = x (16mx+i), k = 8*g + j ; g,j -> rho=16s+4g+(j&3), part=j>>2
                A2=np.zeros((16,32)); B2=np.zeros((32,16))
                for g in range(4):
                    for j in range(8):
                        k=8*g+j; rr=4*g+(j&3)
                        vals=D[s][rr,:]  # over x (i)
                        b=(vals>>8)&255 if j>>2 else vals&255
                        A2[:,k]=b*2.0**-24
                        for jj in range(16): B2[k,jj]=col[dd,jj+16*g,j]
                acc+=A2@B2
            # acc[i][j]: x=16mx+i, y=16ny+j
            out[16*ny:16*ny+16,16*mx:16*mx+16]=acc.T
    got=np.clip(np.round(out[:37,:40]*64),0,255)
    assert (got == ref).all(), trial
print("ok")
