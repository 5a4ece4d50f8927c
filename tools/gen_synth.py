"""Synthetic 8-bit 4:2:0 test content: textured scene with sub-pixel pan, optional zoom,
a moving sine ramp and N(0,2) noise, seed 1234.  Usage: gen_synth.py W H FRAMES OUT.yuv [ZOOM] [VIDEO_RANGE] [FADE]
VIDEO_RANGE=1 maps luma into [16, 235] like broadcast content: the reference encoder's LMCS analysis
(EncReshape::preAnalyzerLMCS) then keeps the reshaper on (full-range content switches it off).
MODE (8th argument) selects content that steers the reference encoder into tools the plain pan rarely picks:
  layers  a second, independently moving textured layer cut by diagonal polygon edges, with a slowly
          changing shading gradient inside the objects (occlusion edges -> GEO, blended
          intra/inter regions -> CIIP);
  screen  screen-like content: flat-coloured panels, one-pixel strokes and glyph rows that scroll by
          whole samples (horizontal / vertical structure -> transform skip and BDPCM).
The YUV is encoded by the reference EncoderApp (tools/encode_streams.sh) into the test bitstreams."""
import numpy as np, sys
W,H,N,out=int(sys.argv[1]),int(sys.argv[2]),int(sys.argv[3]),sys.argv[4]
ZOOM=float(sys.argv[5]) if len(sys.argv)>5 else 0.002
VR=len(sys.argv)>6 and sys.argv[6]=='1'
FADE=float(sys.argv[7]) if len(sys.argv)>7 else 0.0   # per-frame luma gain step (weighted-prediction content)
MODE=sys.argv[8] if len(sys.argv)>8 else ''
rng=np.random.default_rng(1234)
base=rng.integers(0,256,(H//8+8,W//8+8)).astype(np.float32)
# smooth texture via upsampling + blur
from numpy import kron
tex=kron(base,np.ones((8,8),np.float32))
k=np.array([1,4,6,4,1],np.float32);k/=k.sum()
for ax in (0,1):
    tex=np.apply_along_axis(lambda v:np.convolve(v,k,'same'),ax,tex)
yy,xx=np.mgrid[0:H,0:W].astype(np.float32)

def sample(t2,X,Y):
    X=np.clip(X,0,t2.shape[1]-2);Y=np.clip(Y,0,t2.shape[0]-2)
    x0=X.astype(int);y0=Y.astype(int);fx=X-x0;fy=Y-y0
    return (t2[y0,x0]*(1-fx)*(1-fy)+t2[y0,x0+1]*fx*(1-fy)+t2[y0+1,x0]*(1-fx)*fy+t2[y0+1,x0+1]*fx*fy)

if MODE=='layers':
    # foreground texture: finer grain, higher contrast; objects: convex polygons with edges at many angles
    b2=rng.integers(0,256,(H//4+8,W//4+8)).astype(np.float32)
    tex2=kron(b2,np.ones((4,4),np.float32))
    for ax in (0,1):
        tex2=np.apply_along_axis(lambda v:np.convolve(v,k,'same'),ax,tex2)
    tex2=np.clip(128+(tex2-128)*1.6,0,255)
    nobj=max(6,(W*H)//(90*90))
    objs=[]
    for i in range(nobj):
        cx,cy=rng.uniform(0,W),rng.uniform(0,H); r=rng.uniform(24,72); nv=int(rng.integers(3,7))
        ang=np.sort(rng.uniform(0,2*np.pi,nv)); vx,vy=rng.uniform(-2.6,2.6),rng.uniform(-1.8,1.8)
        objs.append((cx,cy,r,ang,vx,vy))
    def poly_mask(cx,cy,r,ang):
        m=np.ones((H,W),bool)
        px=cx+r*np.cos(ang); py=cy+r*np.sin(ang)
        for j in range(len(ang)):
            x1,y1,x2,y2=px[j],py[j],px[(j+1)%len(ang)],py[(j+1)%len(ang)]
            m&=((x2-x1)*(yy-y1)-(y2-y1)*(xx-x1))>=0
        return m

if MODE=='screen':
    srng=np.random.default_rng(4321)
    canvas=np.full((H+64,W+64),230,np.float32)
    for i in range((W*H)//900):   # flat panels
        x0,y0=srng.integers(0,W+40),srng.integers(0,H+40); w,h=srng.integers(8,96),srng.integers(8,64)
        canvas[y0:y0+h,x0:x0+w]=srng.choice([30,60,90,128,170,200,250])
    for i in range((W*H)//200):   # glyph rows: one-pixel strokes
        x0,y0=srng.integers(0,W+56),srng.integers(0,H+56); g=srng.integers(0,2,(7,5))
        for gy in range(7):
            for gx in range(5):
                if g[gy,gx]: canvas[y0+gy,x0+gx]=srng.choice([0,20,255])
    for i in range(H//16):        # ruled lines
        y0=srng.integers(0,H+60); canvas[y0,:]=srng.choice([0,255])
        x0=srng.integers(0,W+60); canvas[:,x0]=srng.choice([0,255])

with open(out,'wb') as f:
  for t in range(N):
    dx,dy=0.37*t*3,0.21*t*3
    s=1.0+ZOOM*t
    X=np.clip((xx-W/2)/s+W/2+dx+16,0,tex.shape[1]-2);Y=np.clip((yy-H/2)/s+H/2+dy+16,0,tex.shape[0]-2)
    x0=X.astype(int);y0=Y.astype(int);fx=X-x0;fy=Y-y0
    v=(tex[y0,x0]*(1-fx)*(1-fy)+tex[y0,x0+1]*fx*(1-fy)+tex[y0+1,x0]*(1-fx)*fy+tex[y0+1,x0+1]*fx*fy)
    v+= 20*np.sin(xx/37.0+t*0.3)+rng.normal(0,2,(H,W))
    if MODE=='layers':
        for (cx,cy,r,ang,vx,vy) in objs:
            ox,oy=cx+vx*t,cy+vy*t
            m=poly_mask(ox,oy,r,ang)
            fg=sample(tex2,xx-vx*t+8,yy-vy*t+8)+ (xx-ox)*0.25*np.sin(t*0.4)+(yy-oy)*0.2*np.cos(t*0.3)
            v=np.where(m,fg,v)
    if MODE=='screen':
        sx,sy=(2*t)%48,(t//2)%48
        v=canvas[sy:sy+H,sx:sx+W].copy()
    if FADE: v=v*(1.0-FADE*t)+12.0*FADE*t*10
    if VR: v=16+np.clip(v,0,255)*(219.0/255.0)
    y=np.clip(v,0,255).astype(np.uint8)
    c=y[::2,::2].astype(np.float32)
    u=np.clip(128+(c-128)*0.25,0,255).astype(np.uint8); w=np.clip(128-(c-128)*0.2,0,255).astype(np.uint8)
    f.write(y.tobytes());f.write(u.tobytes());f.write(w.tobytes())
