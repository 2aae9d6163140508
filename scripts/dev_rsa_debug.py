import sys; sys.path.insert(0,'mochi-db_amd'); sys.path.insert(0,'tests')
import numpy as np, oracle_ffi as O, workload as W, mochi_hip as mh
L=74; B=28; MASK=(1<<B)-1
pems=W.load_keys(2); mods=[O.pem_modulus(p) for p in pems]
sigs=[]; signer=[]
for i in range(6):
    k=i%2; msg=W.encode_grant(f"k{i}",5+i,"a"*128); sigs.append(O.rsa_sign(pems[k],msg)); signer.append(k)
ver=mh.Verifier(mods,0)
y,z=mh.rsa_public_op(ver, np.frombuffer(b"".join(sigs),np.uint8), np.array(signer), want_z=True)
for i in range(6):
    N=int.from_bytes(mods[signer[i]],'big'); s=int.from_bytes(sigs[i],'big'); R=1<<(B*L)
    ye=pow(s,65537,N); yg=int.from_bytes(y[i].tobytes(),'big')
    zg=sum(int(v)<<(B*j) for j,v in enumerate(z[i]))
    ze=(pow(s,65536,N)*pow(pow(R,65535,N),-1,N))%N
    print(i, 'y ok', yg==ye, 'z ok', zg%N==ze, 'z<2n', zg<2*N, hex(yg)[:40], hex(ye)[:40])
    print('   zg limbs', [hex(int(v)) for v in z[i][:4]], 'ze', [hex((ze>>(B*j))&MASK) for j in range(4)])
