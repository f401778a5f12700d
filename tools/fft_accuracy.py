"""Float32 accuracy of the two 256-point complex FFT formulations used on the GPU, emulated in numpy
(one rounding per operation, no FMA): the radix-4 Stockham ping-pong (spectral.hip fft256, the debug
k_stft / k_istft path) and the register four-step 16 x 16 (fft_common.h dft16 + stft.hip / istft.hip),
both against a float64 FFT on 2000 random frames. DESIGN.md section 4d.

usage: python tools/fft_accuracy.py   (a few seconds on the CPU)
"""
import numpy as np
f32=np.float32
rng=np.random.default_rng(0)
NF=2000
z=(rng.standard_normal((NF,256))+1j*rng.standard_normal((NF,256))).astype(np.complex64)
ref=np.fft.fft(z.astype(np.complex128),axis=1)
tw=np.exp(-2j*np.pi*np.arange(512)/512).astype(np.complex64)
def cm(a,b): return (a*b).astype(np.complex64)
def stockham(x):
    x=x.copy()
    for Ns in [1,4,16,64]:
        out=np.empty_like(x)
        for j in range(64):
            k=j&(Ns-1)
            v=[x[:,j+r*64] for r in range(4)]
            if Ns>1:
                for r in range(1,4):
                    v[r]=cm(v[r],tw[2*((r*k*(64//Ns))&255)])
            a0=v[0]+v[2]; a1=v[0]-v[2]; a2=v[1]+v[3]; a3=v[1]-v[3]
            a3=(a3.imag-1j*a3.real).astype(np.complex64)
            idx=(j//Ns)*Ns*4+k
            out[:,idx]=a0+a2; out[:,idx+Ns]=a1+a3; out[:,idx+2*Ns]=a0-a2; out[:,idx+3*Ns]=a1-a3
        x=out
    return x
C1=f32(0.9238795042037964); S1=f32(0.3826834261417389); R=f32(0.7071067690849304)
W16={1:(C1,S1),2:(R,R),3:(S1,C1),6:(-R,R),9:(-C1,-S1)}
def dft4(v0,v1,v2,v3):
    s0=v0+v2; d0=v0-v2; s1=v1+v3; d1=v1-v3
    d1=(d1.imag-1j*d1.real).astype(np.complex64)
    return s0+s1, d0+d1, s0-s1, d0-d1
def d16(k): return (k>>2)+4*(k&3)
def dft16(x):
    x=list(x)
    for na in range(4):
        x[na],x[na+4],x[na+8],x[na+12]=dft4(x[na],x[na+4],x[na+8],x[na+12])
    for na in range(1,4):
        for kb in range(1,4):
            p=na*kb
            if p==4: x[na+4*kb]=(x[na+4*kb].imag-1j*x[na+4*kb].real).astype(np.complex64)
            else:
                c,s=W16[p]; x[na+4*kb]=cm(x[na+4*kb],np.complex64(c-1j*s))
    for kb in range(4):
        x[4*kb],x[4*kb+1],x[4*kb+2],x[4*kb+3]=dft4(x[4*kb],x[4*kb+1],x[4*kb+2],x[4*kb+3])
    return x
def fourstep(z):
    out=np.empty_like(z)
    A=np.empty((NF,16,16),np.complex64)  # A[k1][c]
    for c in range(16):
        x=[z[:,16*n1+c] for n1 in range(16)]
        x=dft16(x)
        for k1 in range(16):
            v=x[d16(k1)]
            if k1>0:
                idx=2*c*k1
                w=tw[idx&255]*(1 if idx<256 else -1)
                v=cm(v,np.complex64(w))
            A[:,k1,c]=v
    for k1 in range(16):
        x=[A[:,k1,n2] for n2 in range(16)]
        x=dft16(x)
        for k2 in range(16): out[:,k1+16*k2]=x[d16(k2)]
    return out
for name,fn in [("stockham",stockham),("fourstep",fourstep)]:
    y=fn(z)
    e=np.abs(y-ref)
    print(name, "max abs err", e.max(), "rms", np.sqrt((e**2).mean()))
