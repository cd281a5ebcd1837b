import sys
integ = sys.argv[1]; W=int(sys.argv[2]); H=int(sys.argv[3]); spp=int(sys.argv[4]); thr=int(sys.argv[5]); out=sys.argv[6]
def quad(p0,p1,p2,p3): return [p0,p1,p2,p3],[(0,1,2),(0,2,3)]
def box(cx,cz,sx,sz,h):
    x0,x1,z0,z1=cx-sx,cx+sx,cz-sz,cz+sz
    v=[(x0,0,z0),(x1,0,z0),(x1,0,z1),(x0,0,z1),(x0,h,z0),(x1,h,z0),(x1,h,z1),(x0,h,z1)]
    f=[(4,5,6),(4,6,7),(0,1,5),(0,5,4),(1,2,6),(1,6,5),(2,3,7),(2,7,6),(3,0,4),(3,4,7),(0,2,1),(0,3,2)]
    return v,f
meshes=[]
meshes.append(("white",)+quad((-1,0,-1),(1,0,-1),(1,0,1),(-1,0,1)))
meshes.append(("white",)+quad((-1,2,-1),(-1,2,1),(1,2,1),(1,2,-1)))
meshes.append(("white",)+quad((-1,0,1),(1,0,1),(1,2,1),(-1,2,1)))
meshes.append(("red",)+quad((-1,0,-1),(-1,0,1),(-1,2,1),(-1,2,-1)))
meshes.append(("green",)+quad((1,0,-1),(1,2,-1),(1,2,1),(1,0,1)))
meshes.append(("white",)+box(-0.35,0.3,0.3,0.3,1.2))
meshes.append(("white",)+box(0.4,-0.3,0.3,0.3,0.6))
meshes.append(("lightm",)+quad((-0.25,1.98,-0.25),(-0.25,1.98,0.25),(0.25,1.98,0.25),(0.25,1.98,-0.25)))
o=['<?xml version="1.0"?>','<scene type="triangle">']
def mat(n,r,g,b): o.append(f'<material name="{n}"><type sval="shinydiffusemat"/><color r="{r}" g="{g}" b="{b}" a="1"/></material>')
mat("white",0.8,0.8,0.8); mat("red",0.8,0.1,0.1); mat("green",0.1,0.8,0.1)
o.append('<material name="lightm"><type sval="light_mat"/><color r="1" g="1" b="1" a="1"/><power fval="10"/></material>')
nt=0
for m,v,f in meshes:
    o.append(f'<mesh vertices="{len(v)}" faces="{len(f)}" has_orco="false" has_uv="false" type="0">')
    for p in v: o.append(f'<p x="{p[0]}" y="{p[1]}" z="{p[2]}"/>')
    o.append(f'<set_material sval="{m}"/>')
    for a,b,c in f: o.append(f'<f a="{a}" b="{b}" c="{c}"/>')
    nt+=len(f)
    o.append('</mesh>')
o.append('<light name="area"><type sval="arealight"/><corner x="-0.25" y="1.979" z="-0.25"/><point1 x="0.25" y="1.979" z="-0.25"/><point2 x="-0.25" y="1.979" z="0.25"/><color r="1" g="1" b="1" a="1"/><power fval="10"/><samples ival="4"/></light>')
o.append(f'<camera name="cam"><type sval="perspective"/><from x="0" y="1" z="-3.6"/><to x="0" y="1" z="0"/><up x="0" y="2" z="-3.6"/><resx ival="{W}"/><resy ival="{H}"/><focal fval="1.3"/></camera>')
if integ=="directlighting":
    o.append('<integrator name="surf"><type sval="directlighting"/><raydepth ival="2"/></integrator>')
else:
    o.append('<integrator name="surf"><type sval="pathtracing"/><raydepth ival="2"/><path_samples ival="1"/><bounces ival="4"/><caustic_type sval="none"/></integrator>')
o.append('<integrator name="vol"><type sval="none"/></integrator>')
o.append(f'<render><camera_name sval="cam"/><integrator_name sval="surf"/><volintegrator_name sval="vol"/><width ival="{W}"/><height ival="{H}"/><AA_minsamples ival="{spp}"/><AA_passes ival="1"/><threads ival="{thr}"/><filter_type sval="box"/><AA_pixelwidth fval="1.0"/><tile_size ival="32"/></render>')
o.append('</scene>')
open(out,'w').write("\n".join(o)+"\n"); print("tris",nt, file=sys.stderr)
