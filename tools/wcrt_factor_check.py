"""Algebra check for the factored W-CRT: the forward through 771 = 3 x 257 and the
inverse via a 771-point interpolation reduced mod Phi_771 both reproduce the dense V / V^-1 product mod q.
Pure Python, one reference modulus, random input.  Dev tool: python3 tools/wcrt_factor_check.py"""
import random
q = 17182765057
def find_eta(q):
    p=771; e=(q-1)//p
    for g in range(2,q):
        eta=pow(g,e,q)
        if eta==1: continue
        if pow(eta,p,q)!=1: continue
        if pow(eta,p//3,q)==1: continue
        if pow(eta,p//257,q)==1: continue
        return eta
eta=find_eta(q)
exp=[(a*257+b*3)%771 for a in (1,2) for b in range(1,257)]
x=[random.randrange(q) for _ in range(512)]
ref=[sum(pow(eta,e*r,q)*x[r] for r in range(512))%q for e in exp]
om=pow(eta,257,q); ze=pow(eta,3,q)
c1=[[pow(om,(ap+1)*r1,q) for r1 in range(3)] for ap in range(2)]
c2=[[pow(om,(ap+1)*((r1+2)%3),q) for r1 in range(3)] for ap in range(2)]
out=[]
for ap in range(2):
    D=[(c1[ap][r2%3]*x[r2] + (c2[ap][r2%3]*x[r2+257] if r2+257<512 else 0))%q for r2 in range(257)]
    for i in range(256):
        s=D[0]+sum(pow(ze,(i+1)*(k+1),q)*D[k+1] for k in range(256))
        out.append(s%q)
print("forward factored == dense:", out == ref)
# inverse
y=ref  # values at the 512 points
inv771=pow(771,q-2,q)
E=[[0]*257 for _ in range(2)]
for ap in range(2):
    for r2 in range(1,257):
        E[ap][r2]=sum(pow(ze,(q-1-0)*0+((-(b+1)*r2)%257),q)*y[ap*256+b] for b in range(256))%q
    E[ap][0]=(-sum(E[ap][1:]))%q
def g(r):
    r1,r2=r%3,r%257
    return inv771*sum(pow(om,(-(ap+1)*r1)%3,q)*E[ap][r2] for ap in range(2))%q
# h = g mod (x^514+x^257+1)
h=[(g(j)-g(j+514))%q for j in range(257)]+[(g(257+j)-g(514+j))%q for j in range(257)]
# Phi_771 coefficients: (x^514+x^257+1)/(x^2+x+1)
num=[0]*515; num[0]=1; num[257]=1; num[514]=1
phi=[0]*513
rem=num[:]
for d in range(514,1,-1):
    c=rem[d]
    if c:
        phi[d-2]=c
        rem[d]-=c; rem[d-1]-=c; rem[d-2]-=c
assert all(v==0 for v in rem)
assert set(phi) <= {-1, 0, 1} and phi[512] == 1
c1q=h[513]; c0q=(h[512]-c1q*phi[511])%q
f=[(h[r]-c0q*phi[r]-(c1q*phi[r-1] if r>0 else 0))%q for r in range(512)]
chk=[sum(pow(eta,e*r,q)*f[r] for r in range(512))%q for e in exp]
print("inverse: V f == y:", chk == y, " f == x:", f == x)
# the factored inverse as gemm.hip computes it: E_a[r2] (r2 = 1..256) from the 256 x 256 GEMM with
# Zi[i][k] = zeta^-((i+1)(k+1)); E_a[0], E_a[255], E_a[256] also by dot products in the digitize kernel;
# h_r2 = sum_a lam1[a][r2 % 3] E_a[r2], h_(r2+257) = sum_a lam2[a][r2 % 3] E_a[r2]; f_j = h_j - c0 phi_j - c1 phi_(j-1)
kap=[[inv771*pow(om,(-(ap+1)*t)%3,q)%q for t in range(3)] for ap in range(2)]
lam1=[[(kap[ap][t]-kap[ap][(t+1)%3])%q for t in range(3)] for ap in range(2)]
lam2=[[(kap[ap][(t+2)%3]-kap[ap][(t+1)%3])%q for t in range(3)] for ap in range(2)]
zi=pow(ze,256,q)
EE=[[sum(pow(zi,(r2*(b+1))%257,q)*y[ap*256+b] for b in range(256))%q for r2 in range(257)] for ap in range(2)]
hh=[0]*514
for r2 in range(257):
    t=r2%3
    hh[r2]=sum(lam1[ap][t]*EE[ap][r2] for ap in range(2))%q
    hh[r2+257]=sum(lam2[ap][t]*EE[ap][r2] for ap in range(2))%q
print("inverse h via lambda == h:", hh == h)
cc1=hh[513]; cc0=(hh[512]-cc1*phi[511])%q
ff=[(hh[j]-cc0*phi[j]-(cc1*phi[j-1] if j>0 else 0))%q for j in range(512)]
print("inverse via lambda: f == x:", ff == x)
