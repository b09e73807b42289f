// dropin.go — the interface-preserving drop-in types (SURVEY.md §8(b) (i)-(iii)).
//
//   - Recorder: descriptor-recording constructors. go-pbrt keeps every scene
//     parameter in unexported fields (Sphere.radius sphere.go:14,
//     GeometricPrimitive.material primitive.go:24, Point.pLight point.go:15,
//     Stratified.xPixelSamples stratified.go:8), so each Recorder method calls
//     the reference constructor AND records its arguments into a SceneBuilder.
//     A scene that uses a type the Recorder never saw marks it Unknown, and
//     Path.RenderFrame then falls back to the CPU render.
//   - Path: satisfies pbrt.Integrator (pkg/pbrt/integrator.go:12-21). Li,
//     Preprocess, GetSampler, GetCamera, SpecularReflect/Transmit are the CPU
//     integrator.Path's (embedded); RenderFrame renders the frame on the GPU
//     and is what the pbrt.Render hook calls (patches/0001-*.patch).
//   - BVH: satisfies pbrt.Aggregate (pkg/pbrt/primitive.go:9-20). Intersect,
//     IntersectP, WorldBound, ... are the CPU accelerator.BVH's (embedded);
//     IntersectBatch / IntersectPBatch run pbrt_gpu_intersect[_p] over ray batches
//     (bvh.go:659-765 semantics, one cgo call per batch).
//
// Not compiled here (no Go toolchain in this image): tests/test_go_shim.py
// checks every C identifier used below against include/pbrt_gpu.h and
// include/pbrt_scene.h.
package pbrtgpu

// #include <stdlib.h>
// #include "pbrt_gpu.h"
// #include "pbrt_scene.h"
import "C"

import (
	"context"
	"errors"
	"fmt"
	"sync"
	"unsafe"

	"github.com/ssttuu/go-pbrt/pkg/accelerator"
	"github.com/ssttuu/go-pbrt/pkg/integrator"
	"github.com/ssttuu/go-pbrt/pkg/lights"
	"github.com/ssttuu/go-pbrt/pkg/materials"
	"github.com/ssttuu/go-pbrt/pkg/pbrt"
	"github.com/ssttuu/go-pbrt/pkg/sampler"
	"github.com/ssttuu/go-pbrt/pkg/shapes"
	"github.com/ssttuu/go-pbrt/pkg/textures"
)

// ------------------------------------------------------------- recorder

// GoTransform copies a pbrt.Transform (transform.go:144-146) into the C
// descriptor: the Go host's own matrices, so the Go-side composition quirks
// (SURVEY §9 #18) reach the device unchanged.
func GoTransform(t *pbrt.Transform) Transform {
	var out Transform
	for i := 0; i < 4; i++ {
		for j := 0; j < 4; j++ {
			out.m.m[i][j] = C.double(t.Matrix[i][j])
			out.m_inv.m[i][j] = C.double(t.MatrixInverse[i][j])
		}
	}
	return out
}

type primRec struct {
	shape, material int
	xform           *Transform // TransformedPrimitive's primToWorld, or nil
}

// Recorder builds the reference's objects and their C descriptor side by side.
type Recorder struct {
	sb       *SceneBuilder
	shapes   map[pbrt.Shape]int
	mats     map[pbrt.Material]int
	prims    map[pbrt.Primitive]primRec
	lights   map[pbrt.Light]C.pbrt_light_desc
	order    []pbrt.Primitive // NewBVH's input order
	maxPrims int
	built    bool
	// Unknown is set when a primitive, material or light reached NewBVH /
	// NewScene without going through the recorder: the GPU cannot describe it.
	Unknown bool
}

func NewRecorder() *Recorder {
	return &Recorder{
		sb:     NewSceneBuilder(),
		shapes: map[pbrt.Shape]int{},
		mats:   map[pbrt.Material]int{},
		prims:  map[pbrt.Primitive]primRec{},
		lights: map[pbrt.Light]C.pbrt_light_desc{},
	}
}

// NewSphereShape is pbrt.NewSphereShape (sphere.go:34-36).
func (r *Recorder) NewSphereShape(name string, o2w *pbrt.Transform, reverse bool, radius float64) pbrt.Shape {
	s := pbrt.NewSphereShape(name, o2w, reverse, radius)
	r.shapes[s] = r.sb.AddSphere(GoTransform(o2w), reverse, radius, -radius, radius, 360)
	return s
}

// NewSphere is pbrt.NewSphere (sphere.go:19-32) with its world-to-object the
// inverse of o2w (as NewSphereShape builds it).
func (r *Recorder) NewSphere(name string, o2w *pbrt.Transform, reverse bool, radius, zMin, zMax, phiMax float64) pbrt.Shape {
	s := pbrt.NewSphere(name, o2w, o2w.Inverse(), reverse, radius, zMin, zMax, phiMax)
	r.shapes[s] = r.sb.AddSphere(GoTransform(o2w), reverse, radius, zMin, zMax, phiMax)
	return s
}

// NewDisk is shapes.NewDisk (pkg/shapes/disk.go:22-35).
func (r *Recorder) NewDisk(o2w *pbrt.Transform, height, radius, inner, phiMax float64) pbrt.Shape {
	s := shapes.NewDisk(o2w, height, radius, inner, phiMax)
	r.shapes[s] = r.sb.AddDisk(GoTransform(o2w), height, radius, inner, phiMax)
	return s
}

// NewMatte is materials.NewMatteMaterial (matte.go:13-19) with a constant Kd
// and sigma (sigma != 0: OrenNayar).
func (r *Recorder) NewMatte(kd [3]float64, sigma float64) pbrt.Material {
	m := materials.NewMatteMaterial(pbrt.NewConstantSpectrumTexture(pbrt.NewRGBSpectrum(kd[0], kd[1], kd[2])),
		pbrt.NewConstantFloatTexture(sigma), nil)
	r.mats[m] = r.sb.AddMatte(kd, sigma)
	return m
}

// NewCheckerMatte is NewMatteMaterial over textures.NewCheckerboard2D(
// pbrt.NewPlanarMapping2D(vs, vt, ds, dt), tex1, tex2) with constant sub-textures
// (server.go:74-79).
func (r *Recorder) NewCheckerMatte(vs, vt [3]float64, ds, dt float64, tex1, tex2 [3]float64, sigma float64) pbrt.Material {
	chk := textures.NewCheckerboard2D(
		pbrt.NewPlanarMapping2D(&pbrt.Vector3f{X: vs[0], Y: vs[1], Z: vs[2]}, &pbrt.Vector3f{X: vt[0], Y: vt[1], Z: vt[2]}, ds, dt),
		pbrt.NewConstantSpectrumTexture(pbrt.NewRGBSpectrum(tex1[0], tex1[1], tex1[2])),
		pbrt.NewConstantSpectrumTexture(pbrt.NewRGBSpectrum(tex2[0], tex2[1], tex2[2])))
	m := materials.NewMatteMaterial(chk, pbrt.NewConstantFloatTexture(sigma), nil)
	r.mats[m] = r.sb.AddCheckerMatte(vs, vt, ds, dt, tex1, tex2, sigma)
	return m
}

// NewMirror is materials.NewMirror (mirror.go:9-14: Kr 0.9).
func (r *Recorder) NewMirror() pbrt.Material {
	m := materials.NewMirror()
	r.mats[m] = r.sb.AddMirror([3]float64{0.9, 0.9, 0.9})
	return m
}

// NewGlass is materials.NewGlass (glass.go:15-26) with constant textures.
func (r *Recorder) NewGlass(kr, kt [3]float64, uRough, vRough, eta float64) pbrt.Material {
	m := materials.NewGlass(pbrt.NewConstantSpectrumTexture(pbrt.NewRGBSpectrum(kr[0], kr[1], kr[2])),
		pbrt.NewConstantSpectrumTexture(pbrt.NewRGBSpectrum(kt[0], kt[1], kt[2])),
		pbrt.NewConstantFloatTexture(uRough), pbrt.NewConstantFloatTexture(vRough), pbrt.NewConstantFloatTexture(eta), nil)
	r.mats[m] = r.sb.AddGlass(kr, kt, uRough, vRough, eta)
	return m
}

// NewGeometricPrimitive is pbrt.NewGeometricPrimitive (primitive.go:29-36).
func (r *Recorder) NewGeometricPrimitive(shape pbrt.Shape, m pbrt.Material) *pbrt.GeometricPrimitive {
	p := pbrt.NewGeometricPrimitive(shape, m)
	si, okS := r.shapes[shape]
	mi, okM := r.mats[m]
	if okS && okM {
		r.prims[p] = primRec{shape: si, material: mi}
	}
	return p
}

// NewTransformedPrimitive is pbrt.NewTransformedPrimitive(p, NewAnimatedTransform(
// p2w, p2w, 0, 1)) (primitive.go:82-87, server.go:56-58): a static transform.
func (r *Recorder) NewTransformedPrimitive(p *pbrt.GeometricPrimitive, p2w *pbrt.Transform) pbrt.Primitive {
	tp := pbrt.NewTransformedPrimitive(p, pbrt.NewAnimatedTransform(p2w, p2w, 0, 1))
	if inner, ok := r.prims[p]; ok {
		x := GoTransform(p2w)
		r.prims[tp] = primRec{shape: inner.shape, material: inner.material, xform: &x}
	}
	return tp
}

// NewBVH is accelerator.NewBVH (bvh.go:223-265) returning the drop-in BVH; the
// GPU scene gets the same primitives in the same order, and the descriptor's
// own BVH build restates NewBVH (truncated SAH, Lomuto partition, §9 #21).
func (r *Recorder) NewBVH(prims []pbrt.Primitive, maxPrimsInNode int, split accelerator.SplitMethod) *BVH {
	r.order = append([]pbrt.Primitive(nil), prims...)
	r.maxPrims = maxPrimsInNode
	if split != accelerator.SplitSAH {
		r.Unknown = true
	}
	for _, p := range prims {
		rec, ok := r.prims[p]
		if !ok {
			r.Unknown = true
			continue
		}
		r.sb.AddPrimitive(rec.shape, rec.material, rec.xform)
	}
	return &BVH{BVH: accelerator.NewBVH(prims, maxPrimsInNode, split), rec: r}
}

// NewPoint is lights.NewPoint (point.go:19-30).
func (r *Recorder) NewPoint(l2w *pbrt.Transform, I [3]float64) pbrt.Light {
	l := lights.NewPoint(l2w, nil, pbrt.NewRGBSpectrum(I[0], I[1], I[2]))
	var d C.pbrt_light_desc
	x := GoTransform(l2w)
	C.pbrt_make_point_light(&x, d3(I), &d)
	r.lights[l] = d
	return l
}

// NewDistant is lights.NewDistant (distant.go:19-26); Preprocess's world radius
// is filled in by the descriptor build (pbrt_sb_build, as NewScene runs it).
func (r *Recorder) NewDistant(l2w *pbrt.Transform, L, w [3]float64) pbrt.Light {
	l := lights.NewDistant(l2w, pbrt.NewRGBSpectrum(L[0], L[1], L[2]), &pbrt.Vector3f{X: w[0], Y: w[1], Z: w[2]})
	var d C.pbrt_light_desc
	x := GoTransform(l2w)
	C.pbrt_make_distant_light(&x, d3(L), d3(w), &d)
	r.lights[l] = d
	return l
}

// NewDiffuseAreaLight is lights.NewDiffuseAreaLight (diffuse.go:17-25) over a
// recorded sphere shape.
func (r *Recorder) NewDiffuseAreaLight(l2w *pbrt.Transform, Le [3]float64, nSamples int32, shape pbrt.Shape, twoSided bool) pbrt.Light {
	l := lights.NewDiffuseAreaLight(l2w, nil, pbrt.NewRGBSpectrum(Le[0], Le[1], Le[2]), nSamples, shape, twoSided)
	si, ok := r.shapes[shape]
	if !ok {
		r.Unknown = true
		return l
	}
	var d C.pbrt_light_desc
	ts := C.int(0)
	if twoSided {
		ts = 1
	}
	C.pbrt_make_diffuse_area_light(d3(Le), C.int(si), ts, &d)
	r.lights[l] = d
	return l
}

// NewScene is pbrt.NewScene (scene.go:16-36); the lights enter the descriptor in order.
func (r *Recorder) NewScene(agg pbrt.Aggregate, ls []pbrt.Light) pbrt.Scene {
	for _, l := range ls {
		d, ok := r.lights[l]
		if !ok {
			r.Unknown = true
			continue
		}
		C.pbrt_sb_add_light(r.sb.b, &d)
	}
	return pbrt.NewScene(agg, ls)
}

// NewFilm is pbrt.NewFilm (film.go:42-76) with a BoxFilter of radius (rx, ry).
func (r *Recorder) NewFilm(filename string, w, h int64, crop [4]float64, rx, ry, diagonal, scale, maxLum float64) *pbrt.Film {
	f := pbrt.NewFilm(filename, &pbrt.Point2i{X: w, Y: h},
		&pbrt.Bounds2f{Min: &pbrt.Point2f{X: crop[0], Y: crop[1]}, Max: &pbrt.Point2f{X: crop[2], Y: crop[3]}},
		pbrt.NewBoxFilter(&pbrt.Point2f{X: rx, Y: ry}), diagonal, scale, maxLum)
	cw := [4]C.double{C.double(crop[0]), C.double(crop[1]), C.double(crop[2]), C.double(crop[3])}
	C.pbrt_sb_set_film(r.sb.b, C.int64_t(w), C.int64_t(h), &cw[0], C.double(rx), C.double(ry), C.double(maxLum))
	return f
}

// NewPerspectiveCamera is pbrt.NewPerspectiveCamera(NewAnimatedTransform(c2w, c2w,
// 0, 1), screen, ...) (camera.go:135-165, server.go:152-159); call after NewFilm.
func (r *Recorder) NewPerspectiveCamera(c2w *pbrt.Transform, screen [4]float64, shutterOpen, shutterClose,
	lensRadius, focalDistance, fov float64, film *pbrt.Film) pbrt.Camera {
	cam := pbrt.NewPerspectiveCamera(pbrt.NewAnimatedTransform(c2w, c2w, 0, 1),
		&pbrt.Bounds2f{Min: &pbrt.Point2f{X: screen[0], Y: screen[1]}, Max: &pbrt.Point2f{X: screen[2], Y: screen[3]}},
		shutterOpen, shutterClose, lensRadius, focalDistance, fov, film, nil)
	x := GoTransform(c2w)
	sw := [4]C.double{C.double(screen[0]), C.double(screen[1]), C.double(screen[2]), C.double(screen[3])}
	C.pbrt_sb_set_perspective_camera(r.sb.b, &x, &sw[0], C.double(shutterOpen), C.double(shutterClose),
		C.double(lensRadius), C.double(focalDistance), C.double(fov))
	return cam
}

// Stratified is sampler.NewStratified (stratified.go:12-19) plus its parameters.
type Stratified struct {
	pbrt.Sampler
	X, Y   int32
	Jitter bool
	NDims  int
}

func NewStratified(x, y int32, jitter bool, nDims int) *Stratified {
	return &Stratified{Sampler: sampler.NewStratified(x, y, jitter, nDims), X: x, Y: y, Jitter: jitter, NDims: nDims}
}

// build finalizes the descriptor once (pbrt_sb_build: NewBVH + NewScene).
func (r *Recorder) build() error {
	if r.built {
		return nil
	}
	if r.Unknown {
		return errors.New("pbrtgpu: the scene holds objects the recorder did not build")
	}
	if err := r.sb.Build(r.maxPrims); err != nil {
		return err
	}
	r.built = true
	return nil
}

// ------------------------------------------------------------------ Path

// Path is integrator.NewPath (path.go:10-17) with a GPU RenderFrame.
type Path struct {
	pbrt.Integrator // the CPU integrator.Path: Li, Preprocess, GetSampler, GetCamera, Specular*

	rec    *Recorder
	rd     C.pbrt_render_desc
	device int

	once     sync.Once
	renderer *Renderer
	err      error
}

// NewPath is integrator.NewPath(maxDepth, camera, sampler, pixelBounds,
// rrThreshold, strategy); device is the HIP ordinal the frame renders on.
func (r *Recorder) NewPath(maxDepth int32, camera pbrt.Camera, smp *Stratified, pixelBounds *pbrt.Bounds2i,
	rrThreshold float64, strategy pbrt.LightSampleStrategy, device int) *Path {
	rd := PathDesc(smp.X, smp.Y, smp.Jitter, int32(smp.NDims), maxDepth, rrThreshold, int32(strategy))
	return &Path{
		Integrator: integrator.NewPath(maxDepth, camera, smp, pixelBounds, rrThreshold, strategy),
		rec:        r,
		rd:         rd,
		device:     device,
	}
}

// RenderFrame implements pbrt.FrameRenderer (patches/0001-*.patch): pbrt.Render's
// whole frame (integrator.go:291-350) on the GPU. The device film is the merged
// XYZ sums MergeFilmTile would hold; it is added to the camera's film and written
// with WriteImage(1.0), as pbrt.Render ends. A scene the recorder cannot describe
// renders on the CPU (pbrt.RenderTiles, the reference's own loop).
func (p *Path) RenderFrame(ctx context.Context, scene pbrt.Scene, tileSize int64) error {
	if err := p.rec.build(); err != nil {
		return pbrt.RenderTiles(ctx, p, scene, tileSize)
	}
	p.once.Do(func() { p.renderer, p.err = NewRenderer(p.rec.sb, p.device) })
	if p.err != nil {
		return p.err
	}
	film := p.GetCamera().GetFilm()
	b := film.CroppedPixelBounds
	xyz := make([]float64, (b.Max.X-b.Min.X)*(b.Max.Y-b.Min.Y)*3)
	rd := p.rd
	rd.tile_size = C.int64_t(tileSize)
	if err := p.renderer.RenderFrame(ctx, &rd, xyz); err != nil {
		return err
	}
	film.MergeXYZ(xyz)
	film.WriteImage(1.0)
	return nil
}

// Close releases the device scene.
func (p *Path) Close() {
	if p.renderer != nil {
		p.renderer.Close()
	}
}

// ------------------------------------------------------------------- BVH

// BVH is accelerator.BVH with batch traversal on the GPU.
type BVH struct {
	*accelerator.BVH // per-ray Intersect / IntersectP / WorldBound (bvh.go:653-779)

	rec      *Recorder
	once     sync.Once
	renderer *Renderer
	err      error
	slotPrim []int32 // BVH slot -> index into the NewBVH input (pbrt_sb_prim_order)
}

// Hit is one batch closest-hit result: Intersect's return value, ray.TMax
// after the call, the primitive hit (nil on a miss) and the interaction's
// Point and geometric Normal.
type Hit struct {
	Hit       bool
	TMax      float64
	Primitive pbrt.Primitive
	Point     [3]float64
	Normal    [3]float64
}

func (b *BVH) device() error {
	b.once.Do(func() {
		if b.err = b.rec.build(); b.err != nil {
			return
		}
		n := len(b.rec.order)
		b.slotPrim = make([]int32, n)
		if n > 0 {
			C.pbrt_sb_prim_order(b.rec.sb.b, (*C.int32_t)(unsafe.Pointer(&b.slotPrim[0])), C.int(n))
		}
		b.renderer, b.err = NewRenderer(b.rec.sb, -1)
	})
	return b.err
}

// cArena is one C allocation holding a batch's SoA arrays. cgo forbids passing
// C a Go value that points at Go memory (pbrt_ray_soa / pbrt_hit_soa hold the
// array pointers: with cgocheck=1 the call panics "cgo argument has Go pointer
// to unpinned Go pointer"), so the arrays live in C memory and the structs
// passed to C hold only C pointers. Slices over the C memory are made with the
// fixed-size-array idiom (no unsafe.Slice: go-pbrt builds with Go 1.11).
type cArena struct {
	base unsafe.Pointer
	off  uintptr
}

// maxBatchRays bounds one device batch: its arrays fit the fixed-size-array
// casts below ([1 << 28]float64) and its arena size, n*(14*8+4+1)+128 bytes,
// fits a 32-bit int; IntersectBatch / IntersectPBatch split larger batches.
const maxBatchRays = 1 << 24

func newArena(bytes int) *cArena {
	if bytes < 8 {
		bytes = 8
	}
	return &cArena{base: C.malloc(C.size_t(bytes))}
}

func (a *cArena) take(bytes int) unsafe.Pointer {
	p := unsafe.Pointer(uintptr(a.base) + a.off)
	a.off += (uintptr(bytes) + 7) &^ 7
	return p
}

func (a *cArena) f64(n int) []float64 { return (*[1 << 28]float64)(a.take(8 * n))[:n:n] }
func (a *cArena) i32(n int) []int32   { return (*[1 << 29]int32)(a.take(4 * n))[:n:n] }
func (a *cArena) u8(n int) []uint8    { return (*[1 << 30]uint8)(a.take(n))[:n:n] }
func (a *cArena) free()               { C.free(a.base) }

func cdp(s []float64) *C.double { return (*C.double)(unsafe.Pointer(&s[0])) }

// packRays copies the rays into a pbrt_ray_soa whose arrays are in arena a.
func packRays(a *cArena, rays []*pbrt.Ray) C.pbrt_ray_soa {
	n := len(rays)
	var o, d [3][]float64
	for k := 0; k < 3; k++ {
		o[k], d[k] = a.f64(n), a.f64(n)
	}
	tmax := a.f64(n)
	for i, r := range rays {
		o[0][i], o[1][i], o[2][i] = r.Origin.X, r.Origin.Y, r.Origin.Z
		d[0][i], d[1][i], d[2][i] = r.Direction.X, r.Direction.Y, r.Direction.Z
		tmax[i] = r.TMax
	}
	var soa C.pbrt_ray_soa
	soa.ox, soa.oy, soa.oz = cdp(o[0]), cdp(o[1]), cdp(o[2])
	soa.dx, soa.dy, soa.dz = cdp(d[0]), cdp(d[1]), cdp(d[2])
	soa.tmax = cdp(tmax)
	return soa
}

// IntersectBatch is BVH.Intersect (bvh.go:659-712) for every ray; like the
// per-ray call it shrinks each ray's TMax to the hit distance.
func (b *BVH) IntersectBatch(rays []*pbrt.Ray, hits []Hit) error {
	n := len(rays)
	if len(hits) < n {
		return fmt.Errorf("pbrtgpu: %d hits for %d rays", len(hits), n)
	}
	if n > maxBatchRays { // the arena's slices and its byte count stay in range
		for i := 0; i < n; i += maxBatchRays {
			j := i + maxBatchRays
			if j > n {
				j = n
			}
			if err := b.IntersectBatch(rays[i:j], hits[i:j]); err != nil {
				return err
			}
		}
		return nil
	}
	if n == 0 {
		return nil
	}
	if err := b.device(); err != nil {
		return err
	}
	// rays: 7 doubles; hits: 7 doubles, an int32 and a byte per ray (+ alignment)
	a := newArena(n*(14*8+4+1) + 16*8)
	defer a.free()
	soa := packRays(a, rays)
	hit, tmax, prim := a.u8(n), a.f64(n), a.i32(n)
	var p, nn [3][]float64
	for k := 0; k < 3; k++ {
		p[k], nn[k] = a.f64(n), a.f64(n)
	}
	var hs C.pbrt_hit_soa
	hs.hit = (*C.uint8_t)(unsafe.Pointer(&hit[0]))
	hs.t_max = cdp(tmax)
	hs.prim = (*C.int32_t)(unsafe.Pointer(&prim[0]))
	hs.px, hs.py, hs.pz = cdp(p[0]), cdp(p[1]), cdp(p[2])
	hs.nx, hs.ny, hs.nz = cdp(nn[0]), cdp(nn[1]), cdp(nn[2])
	if rc := C.pbrt_gpu_intersect(b.renderer.ctx, &soa, C.size_t(n), &hs); rc != C.PBRT_OK {
		return fmt.Errorf("pbrt_gpu_intersect: %s", C.GoString(C.pbrt_gpu_last_error(b.renderer.ctx)))
	}
	for i := 0; i < n; i++ {
		hits[i] = Hit{Hit: hit[i] != 0, TMax: tmax[i]}
		rays[i].TMax = tmax[i]
		if hits[i].Hit {
			hits[i].Primitive = b.rec.order[b.slotPrim[prim[i]]]
			hits[i].Point = [3]float64{p[0][i], p[1][i], p[2][i]}
			hits[i].Normal = [3]float64{nn[0][i], nn[1][i], nn[2][i]}
		}
	}
	return nil
}

// IntersectPBatch is BVH.IntersectP (bvh.go:713-765) for every ray.
func (b *BVH) IntersectPBatch(rays []*pbrt.Ray, occluded []bool) error {
	n := len(rays)
	if len(occluded) < n {
		return fmt.Errorf("pbrtgpu: %d results for %d rays", len(occluded), n)
	}
	if n > maxBatchRays {
		for i := 0; i < n; i += maxBatchRays {
			j := i + maxBatchRays
			if j > n {
				j = n
			}
			if err := b.IntersectPBatch(rays[i:j], occluded[i:j]); err != nil {
				return err
			}
		}
		return nil
	}
	if n == 0 {
		return nil
	}
	if err := b.device(); err != nil {
		return err
	}
	a := newArena(n*(7*8+1) + 8*8)
	defer a.free()
	soa := packRays(a, rays)
	occ := a.u8(n)
	if rc := C.pbrt_gpu_intersect_p(b.renderer.ctx, &soa, C.size_t(n), (*C.uint8_t)(unsafe.Pointer(&occ[0]))); rc != C.PBRT_OK {
		return fmt.Errorf("pbrt_gpu_intersect_p: %s", C.GoString(C.pbrt_gpu_last_error(b.renderer.ctx)))
	}
	for i := 0; i < n; i++ {
		occluded[i] = occ[i] != 0
	}
	return nil
}
