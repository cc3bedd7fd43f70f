"""Host check of erf_fast (csrc/mapa_common.h): the two minimax pieces evaluated in float32 with FMAs (emulated in
float64, one rounding), max error in ulp against math.erf over [-6, 6] and 200k normal samples."""
import numpy as np, math
f32=np.float32
def fma(a,b,c): return f32(np.float64(a)*np.float64(b)+np.float64(c))
def erf_j(a):
    a=f32(a); t=f32(abs(a)); s=f32(a*a)
    # large branch
    r=fma(f32(-1.72853470e-5),t,f32(3.83197126e-4))
    u=fma(f32(-3.88396438e-3),t,f32(2.42546219e-2))
    r=fma(r,s,u)
    r=fma(r,t,f32(-1.06777877e-1))
    r=fma(r,t,f32(-6.34846687e-1))
    r=fma(r,t,f32(-1.28717512e-1))
    r=fma(r,t,-t)
    e=f32(np.exp2(np.float64(f32(r*f32(1.4426950408889634)))))
    big=f32(1)-e; big=f32(math.copysign(big,a))
    q=f32(-5.96761703e-4)
    q=fma(q,s,f32(4.99119423e-3))
    q=fma(q,s,f32(-2.67681349e-2))
    q=fma(q,s,f32(1.12819925e-1))
    q=fma(q,s,f32(-3.76125336e-1))
    q=fma(q,s,f32(1.28379166e-1))
    q=fma(q,a,a)
    return big if t>f32(0.927734375) else q
xs=np.concatenate([np.linspace(-6,6,200001), np.random.RandomState(0).randn(200000)*2]).astype(np.float32)
worst=0; wx=None
for x in xs:
    y=erf_j(x); ref=math.erf(float(x))
    ulp=np.spacing(f32(abs(ref))) if ref!=0 else 1e-45
    e=abs(float(y)-ref)/float(ulp)
    if e>worst: worst=e; wx=x
print("max ulp err", worst, "at", wx)
