"""Error band of the reference's f32 ray/3-sigma-ellipsoid discriminant (gaussian.h:137-151) in whitened units, which
sizes the secondary rays' chord band (vr_gauss.hip kChordBand). Gaussians of the make_random distribution
(diameters U(0.01, 0.035), Haar rotations), origins 0.01-3 units away, rays aimed to graze: the f32 discriminant
B*B - 4*A*C (Eigen's evaluation order) divided by 4A against the exact D = 9 - e2 (double, same f32 M, p, d), in
units of eps * c (eps = 2^-23, c = p.M.p). CPU only: python3 tools/chord_band.py"""
import numpy as np
f=np.float32
rng=np.random.default_rng(1)
N=400000
# make_random Gaussians: diameters U(0.01,0.035), Haar rotation
d=rng.uniform(0.01,0.035,(N,3)).astype(np.float64)
A=rng.normal(size=(N,3,3)); Q,Rm=np.linalg.qr(A); Q=Q*np.sign(np.diagonal(Rm,axis1=1,axis2=2))[:,None,:]
det=np.linalg.det(Q); Q[det<0,:,0]*=-1
S=(d/2)**2
cov=np.einsum('nij,nj,nkj->nik',Q,S,Q).astype(np.float32)
M=np.linalg.inv(cov.astype(np.float64)).astype(np.float32)  # approx inverse (bits don't matter for error stats)
# origin at distance r along random direction from mean, direction aimed to graze: pick chord distance
u=rng.normal(size=(N,3)); u/=np.linalg.norm(u,axis=1)[:,None]
dist=10**rng.uniform(-2,0.5,N)  # 0.01 .. 3 units
mean=rng.uniform(-1,1,(N,3)).astype(np.float32)
o=(mean+u*dist[:,None]).astype(np.float32)
# direction: towards mean with random perturbation
v=(mean-o).astype(np.float64); v/=np.linalg.norm(v,axis=1)[:,None]
w=rng.normal(size=(N,3))*rng.uniform(0,0.02,N)[:,None]/np.maximum(dist,0.01)[:,None]
dr=(v+w); dr/=np.linalg.norm(dr,axis=1)[:,None]; dr=dr.astype(np.float32)
def mul(M,x):
    return np.stack([M[:,i,0]*x[:,0]+(M[:,i,1]*x[:,1]+M[:,i,2]*x[:,2]) for i in range(3)],1)
def dot(a,b): return a[:,0]*b[:,0]+(a[:,1]*b[:,1]+a[:,2]*b[:,2])
p=(o-mean).astype(np.float32)
Md=mul(M,dr); Mp=mul(M,p)
Af=dot(dr,Md); Bf=f(2)*dot(p,Md); Cf=dot(p,Mp)-f(9)
disc=Bf*Bf-f(4)*Af*Cf
# exact in double with the same (f32) M, p, d
Md64=np.einsum('nij,nj->ni',M.astype(np.float64),dr.astype(np.float64)); Mp64=np.einsum('nij,nj->ni',M.astype(np.float64),p.astype(np.float64))
A64=(dr*Md64).sum(1); B64=2*(p*Mp64*0+p*Md64).sum(1); C64=(p*Mp64).sum(1)
D64=(B64*B64-4*A64*(C64-9))/(4*A64)
Df=disc.astype(np.float64)/(4*A64)
c=C64
err=np.abs(Df-D64)/c
near=np.abs(D64)<0.05*c
print("samples near", near.sum())
for q in [50,90,99,99.9,99.99,100]:
    print(q, np.percentile(err[near],q))
# relative to eps
eps=2**-23
print("max err/(eps*c)", err[near].max()/eps)
# condition number effect
lam=S; kappa=lam.max(1)/lam.min(1)
print("max err/(eps*c*kappa)", (err/ (eps*kappa))[near].max())
