# probe-only: procedural displaced-sphere mesh (NU x NV grid, 2*NU*(NV-1) tris) inside a Cornell-like box with one area light
import sys, math
NU=int(sys.argv[1]); NV=int(sys.argv[2]); W=int(sys.argv[3]); H=int(sys.argv[4]); spp=int(sys.argv[5]); thr=int(sys.argv[6]); out=sys.argv[7]
o=['<?xml version="1.0"?>','<scene type="triangle">']
o.append('<material name="white"><type sval="shinydiffusemat"/><color r="0.8" g="0.8" b="0.8" a="1"/></material>')
o.append('<material name="red"><type sval="shinydiffusemat"/><color r="0.8" g="0.1" b="0.1" a="1"/></material>')
def mesh(mat,v,f):
    o.append(f'<mesh vertices="{len(v)}" faces="{len(f)}" has_orco="false" has_uv="false" type="0">')
    o.extend(f'<p x="{p[0]:.6f}" y="{p[1]:.6f}" z="{p[2]:.6f}"/>' for p in v)
    o.append(f'<set_material sval="{mat}"/>')
    o.extend(f'<f a="{a}" b="{b}" c="{c}"/>' for a,b,c in f)
    o.append('</mesh>')
mesh("white",[(-3,0,-3),(3,0,-3),(3,0,3),(-3,0,3)],[(0,2,1),(0,3,2)])
v=[];f=[]
for j in range(NV):
    th=math.pi*j/(NV-1)
    for i in range(NU):
        ph=2*math.pi*i/NU
        r=1.0+0.08*math.sin(7*th)*math.cos(9*ph)+0.03*math.sin(23*th+5*ph)
        v.append((r*math.sin(th)*math.cos(ph), 1.2+r*math.cos(th), r*math.sin(th)*math.sin(ph)))
for j in range(NV-1):
    for i in range(NU):
        a=j*NU+i; b=j*NU+(i+1)%NU; c=a+NU; d=b+NU
        f.append((a,c,b)); f.append((b,c,d))
mesh("red",v,f)
o.append('<light name="area"><type sval="arealight"/><corner x="-0.5" y="3" z="-0.5"/><point1 x="0.5" y="3" z="-0.5"/><point2 x="-0.5" y="3" z="0.5"/><color r="1" g="1" b="1" a="1"/><power fval="8"/><samples ival="1"/></light>')
o.append(f'<camera name="cam"><type sval="perspective"/><from x="0" y="1.5" z="-4"/><to x="0" y="1.2" z="0"/><up x="0" y="2.5" z="-4"/><resx ival="{W}"/><resy ival="{H}"/><focal fval="1.4"/></camera>')
o.append('<integrator name="surf"><type sval="pathtracing"/><raydepth ival="2"/><path_samples ival="1"/><bounces ival="3"/><caustic_type sval="none"/></integrator>')
o.append('<integrator name="vol"><type sval="none"/></integrator>')
o.append(f'<render><camera_name sval="cam"/><integrator_name sval="surf"/><volintegrator_name sval="vol"/><width ival="{W}"/><height ival="{H}"/><AA_minsamples ival="{spp}"/><AA_passes ival="1"/><threads ival="{thr}"/><filter_type sval="box"/><AA_pixelwidth fval="1.0"/><tile_size ival="32"/></render>')
o.append('</scene>')
open(out,'w').write("\n".join(o)+"\n"); print("tris",len(f)+2,file=sys.stderr)
