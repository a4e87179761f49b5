"""CPU check of k_mid_tree's climb (rt_lbvh.hip): the Apetrei bottom-up construction with in-block
LDS hand-offs and the split-only "parent stays inside the block" test, run under random thread
interleavings, must give Karras' tree, and every split's two arrivals must make the same decision
(one hand-off place per split). Random sorted key sets, block sizes 4 ... 1024:
  python tools/apetrei_sim.py"""
import random
def clz64(x):
    return 64 - x.bit_length()
def karras(keys):
    n=len(keys); k64=[(keys[i]<<32)|i for i in range(n)]
    def d(i,j):
        if j<0 or j>=n: return -1
        return clz64(k64[i]^k64[j])
    ch={}
    for i in range(n-1):
        dd=1 if d(i,i+1)-d(i,i-1)>=0 else -1
        dmin=d(i,i-dd); lmax=2
        while d(i,i+lmax*dd)>dmin: lmax<<=1
        l=0; t=lmax>>1
        while t>=1:
            if d(i,i+(l+t)*dd)>dmin: l+=t
            t>>=1
        j=i+l*dd; dn=d(i,j); s=0; t=l
        while True:
            t=(t+1)>>1
            if d(i,i+(s+t)*dd)>dn: s+=t
            if t<=1: break
        g=i+s*dd+(dd if dd<0 else 0)
        lo,hi=min(i,j),max(i,j)
        left=('L',g) if lo==g else ('I',g)
        right=('L',g+1) if hi==g+1 else ('I',g+1)
        ch[i]=(left,right,lo,hi)
    # canonical: map internal node -> leaf range
    def canon(node):
        t,x=node
        if t=='L': return ('L',x)
        l,r,lo,hi=ch[x]
        return (canon(l),canon(r))
    return canon(('I',0)) if n>1 else ('L',0)
def apetrei(keys,S,order_seed):
    n=len(keys); k64=[(keys[i]<<32)|i for i in range(n)]
    rng=random.Random(order_seed)
    # each thread a generator that yields at hand-offs; scheduler interleaves randomly
    flags={}; slots={}; bins={}; root=[None]; decisions={}
    def thread(i):
        B=(i//S)*S
        l=r=i; ref=('L',i); local=True
        def key(p): return k64[p]
        while not (l==0 and r==n-1):
            dl=clz64(key(l-1)^key(l)) if l>0 else -1
            dr=clz64(key(r)^key(r+1)) if r<n-1 else -1
            left=dr>dl; s=r if left else l-1; q=dr if left else dl
            pl=local and s>=B and s+1<B+S
            if pl:
                ks=key(s)
                pl=(B==0 or clz64(ks^key(B-1))<q) and (B+S>=n or clz64(ks^key(B+S))<q)
            side=0 if left else 1
            where=('LDS',B) if pl else ('G',)
            decisions.setdefault(s,set()).add(where)
            slots[(where,s,side)]=(ref,l if left else r)
            yield
            old=flags.get((where,s),0); flags[(where,s)]=old+1
            if old==0: return
            oref,ob=slots[(where,s,1-side)]
            lr,rr=(ref,oref) if left else (oref,ref)
            bins[s]=(lr,rr)
            if left: r=ob
            else: l=ob
            ref=('I',s); local=pl
            yield
        root[0]=ref
    ths=[thread(i) for i in range(n)]
    live=list(range(n))
    while live:
        k=rng.randrange(len(live))
        try: next(ths[live[k]])
        except StopIteration: live.pop(k)
    for s,w in decisions.items(): assert len(w)==1,(s,w)
    def canon(node):
        t,x=node
        if t=='L': return ('L',x)
        l,r=bins[x]; return (canon(l),canon(r))
    return canon(root[0])
for trial in range(300):
    rng=random.Random(trial)
    n=rng.randint(2,200)
    bits=rng.choice([2,4,8,30])
    keys=sorted(rng.randrange(1<<bits) for _ in range(n))
    S=rng.choice([4,8,16,64,1024])
    a=karras(keys); b=apetrei(keys,S,trial)
    assert a==b,(trial,n,S)
print("ok")
