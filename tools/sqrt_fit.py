"""Search for the fp32 operation sequence behind a host's torch.sqrt (MKL VML vsSqrt):
Newton-Raphson forms around the hardware rsqrt14 / rsqrt approximations, scored against
tools/sqrt_probe.py output (mismatches on every 7th float of [1, 4); 0 = found).
    python tools/sqrt_fit.py PROBE_DIR"""
import sys; import os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from oracle.geometry_ref import fma32
f32=np.float32
D=sys.argv[1]
d=np.load(D+'/sqrt_offsets.npz')['d'].astype(np.int64)
bits=np.arange(0x3F800000,0x3F800000+(1<<24),dtype=np.uint32)
x=bits.view(f32)
cr=np.sqrt(x.astype(np.float64)).astype(f32)
target=(cr.view(np.int32).astype(np.int64)+d).astype(np.int32).view(f32)
sub=slice(None,None,7)
x=x[sub]; target=target[sub]
tabs={k:np.load(D+'/%s.npz'%k)['a'].view(f32)[sub] for k in ('rsqrt14','rsqrt','rcp14','rcp')}
def fnma(a,b,c): return fma32(-a,b,c)
res={}
for tn in ('rsqrt14','rsqrt'):
    y0=tabs[tn]
    # refine rsqrt first (optional)
    for refine in (0,1):
        y=y0
        if refine:
            # y1 = y0*(1.5 - 0.5*x*y0*y0)
            h=(f32(0.5)*x).astype(f32)
            e=fnma((h*y).astype(f32), y, f32(1.5))
            y=(y*e).astype(f32)
        g=(x*y).astype(f32); h=(f32(0.5)*y).astype(f32)
        r=fnma(g,h,f32(0.5))
        g1=fma32(g,r,g); h1=fma32(h,r,h)
        res[(tn,refine,'g')]=g
        res[(tn,refine,'g1')]=g1
        dd=fnma(g1,g1,x); res[(tn,refine,'g2')]=fma32(dd,h1,g1)
        dd0=fnma(g,g,x); res[(tn,refine,'g0corr')]=fma32(dd0,h,g)
        res[(tn,refine,'g1corr_h')]=fma32(dd,h,g1)
        # Newton on sqrt directly: s = 0.5*(g + x/g)
        res[(tn,refine,'heron')]=(f32(0.5)*(g+(x/g).astype(f32)).astype(f32)).astype(f32)
        # y*x then x*y*(1.5-0.5*x*y*y)
        e2=fnma((f32(0.5)*x*y).astype(f32),y,f32(1.5))
        res[(tn,refine,'xy_e')]=((x*y).astype(f32)*e2).astype(f32)
        res[(tn,refine,'x_ye')]=(x*(y*e2).astype(f32)).astype(f32)
for k,v in sorted(res.items(), key=lambda kv: np.count_nonzero(kv[1]!=target)):
    print(np.count_nonzero(v!=target), len(target), k)
