"""LDS bank-conflict model of the exact fbank's lane program
(catears_amd/csrc/fbank8_ops.h): for each transpose access pattern, the extra
passes per wave-instruction on 64 banks of 4 B (b32: 32 lanes per pass;
b128: 16 lanes per pass, 4 banks each; equal addresses broadcast), summed
over one 8-frame group, for frame strides S and transpose layouts
phys(p) = p + P * (p >> G).  python tools/fb_bank_model.py"""
import sys
kBlk1=[0,2,3,4,6,8,11,14]; kBlk2=[1,5,7,9,13,10,12,15]
def brev3(v): return ((v&1)<<2)|(v&2)|((v>>2)&1)
def brev4(v): return ((v&1)<<3)|((v&2)<<1)|((v>>1)&2)|((v>>3)&1)
def cost(addrs, width):
    lanes_per = 32 if width==1 else 16
    extra=0
    for g in range(0,64,lanes_per):
        banks={}; uniq=set()
        for l in range(g,g+lanes_per):
            a=addrs[l]
            if a in uniq: continue
            uniq.add(a)
            for w in range(width):
                b=(a+w)%64; banks[b]=banks.get(b,0)+1
        extra+=max(banks.values())-1
    return extra
def model(S,P,G):
    phys=lambda p: p + P*(p>>G)
    fb=lambda l: (l>>3)*S
    lanes=range(64)
    t={}
    t['store_a']=2*sum(cost([fb(l)+phys((l&7)+8*j) for l in lanes],1) for j in range(32))
    def pbp(q,j): return 16*(kBlk1[q] if j<16 else kBlk2[q])+(j&15)
    t['ld/st_b']=4*sum(cost([fb(l)+phys(pbp(l&7,j)) for l in lanes],4) for j in range(0,32,4))
    def lp(l,tt,w):
        q=l&7
        if w=='x': p=(brev3(q)<<1)+(brev4(tt+1)<<4) if tt<15 else brev4(q+1)
        else: p=15-(brev3(q)<<1)+240-(brev4(tt)<<4) if tt<15 else brev4(15-q)
        return fb(l)+phys(p)
    t['load_post']=2*sum(cost([lp(l,tt,w) for l in lanes],1) for tt in range(16) for w in 'xy')
    t['post_store']=sum(cost([fb(l)+16*(l&7)+1+tt for l in lanes],1)+cost([fb(l)+240-16*(l&7)+15-tt for l in lanes],1) for tt in range(16))
    return t
res=[]
for S in range(264,276,4):
  for G in (4,5,6,7):
    for P in (0,4,8,12):
      if 255+P*(255>>G) >= S: continue
      t=model(S,P,G); res.append((sum(t.values()),S,P,G,t))
res.sort(key=lambda x:x[0])
for r in res[:12]: print(r)
