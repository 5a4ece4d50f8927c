"""Synthetic 8-bit 4:2:0 test content: textured scene with sub-pixel pan, optional zoom,
a moving sine ramp and N(0,2) noise, seed 1234.  Usage: gen_synth.py W H FRAMES OUT.yuv [ZOOM] [VIDEO_RANGE] [FADE]
VIDEO_RANGE=1 maps luma into [16, 235] like broadcast content: the reference encoder's LMCS analysis
(EncReshape::preAnalyzerLMCS) then keeps the reshaper on (full-range content switches it off).
The YUV is encoded by the reference EncoderApp (tools/encode_streams.sh) into the test bitstreams."""
import numpy as np, sys
W,H,N,out=int(sys.argv[1]),int(sys.argv[2]),int(sys.argv[3]),sys.argv[4]
ZOOM=float(sys.argv[5]) if len(sys.argv)>5 else 0.002
VR=len(sys.argv)>6 and sys.argv[6]=='1'
FADE=float(sys.argv[7]) if len(sys.argv)>7 else 0.0   # per-frame luma gain step (weighted-prediction content)
rng=np.random.default_rng(1234)
base=rng.integers(0,256,(H//8+8,W//8+8)).astype(np.float32)
# smooth texture via upsampling + blur
from numpy import kron
tex=kron(base,np.ones((8,8),np.float32))
k=np.array([1,4,6,4,1],np.float32);k/=k.sum()
for ax in (0,1):
    tex=np.apply_along_axis(lambda v:np.convolve(v,k,'same'),ax,tex)
yy,xx=np.mgrid[0:H,0:W].astype(np.float32)
with open(out,'wb') as f:
  for t in range(N):
    dx,dy=0.37*t*3,0.21*t*3
    s=1.0+ZOOM*t
    X=np.clip((xx-W/2)/s+W/2+dx+16,0,tex.shape[1]-2);Y=np.clip((yy-H/2)/s+H/2+dy+16,0,tex.shape[0]-2)
    x0=X.astype(int);y0=Y.astype(int);fx=X-x0;fy=Y-y0
    v=(tex[y0,x0]*(1-fx)*(1-fy)+tex[y0,x0+1]*fx*(1-fy)+tex[y0+1,x0]*(1-fx)*fy+tex[y0+1,x0+1]*fx*fy)
    v+= 20*np.sin(xx/37.0+t*0.3)+rng.normal(0,2,(H,W))
    if FADE: v=v*(1.0-FADE*t)+12.0*FADE*t*10
    if VR: v=16+np.clip(v,0,255)*(219.0/255.0)
    y=np.clip(v,0,255).astype(np.uint8)
    c=y[::2,::2].astype(np.float32)
    u=np.clip(128+(c-128)*0.25,0,255).astype(np.uint8); w=np.clip(128-(c-128)*0.2,0,255).astype(np.uint8)
    f.write(y.tobytes());f.write(u.tobytes());f.write(w.tobytes())
