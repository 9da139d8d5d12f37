import random
RING=1536; D=4
def sim(sizes):
    head=0; iss=0; red=0; posv={}; inflight={}
    bad=0; fulls=0
    n=len(sizes)
    while red<n:
        while iss<n and iss-red<D:
            A=(sizes[iss]+63)//64*64
            if iss==red:
                pos=head if head+A<=RING else 0
            else:
                old=posv[red]
                if head==old: pos=-1
                elif head>old:
                    pos=head if head+A<=RING else (0 if A<=old else -1)
                else:
                    pos=head if head+A<=old else -1
                if head==old: fulls+=1
            if pos<0: break
            # overlap check vs in-flight
            for j,(p,a) in inflight.items():
                if not (pos+A<=p or p+a<=pos): bad+=1
            inflight[iss]=(pos,A); posv[iss]=pos; head=pos+A; iss+=1
        del inflight[red]; red+=1
    return bad,fulls
random.seed(1)
tb=tf=0
for w in range(2000):
    sizes=[]
    for j in range(40):
        k=random.randint(5,15)
        s=sum(((random.randint(64,1350)+15)//16) for _ in range(k))
        sizes.append(s)
    b,f=sim(sizes); tb+=b; tf+=f
print("overlaps",tb,"full-ambiguous",tf)
def sim2(sizes):
    head=0; iss=0; red=0; posv={}; inflight={}
    n=len(sizes)
    while red<n:
        while iss<n and iss-red<D:
            A=(sizes[iss]+63)//64*64
            if iss==red:
                pos=head if head+A<=RING else 0
            else:
                old=posv[red]
                if head==old: pos=-1
                elif head>old:
                    pos=head if head+A<=RING else (0 if A<=old else -1)
                else:
                    pos=head if head+A<=old else -1
            if pos<0: break
            for j,(p,a) in inflight.items():
                if not (pos+A<=p or p+a<=pos):
                    print("overlap: new", iss, (pos,A), "with", j, (p,a), "red",red,"head",head,"inflight",inflight); return
            inflight[iss]=(pos,A); posv[iss]=pos; head=pos+A; iss+=1
        del inflight[red]; red+=1
random.seed(1)
for w in range(50):
    sizes=[]
    for j in range(40):
        k=random.randint(5,15)
        sizes.append(sum(((random.randint(64,1350)+15)//16) for _ in range(k)))
    sim2(sizes)
