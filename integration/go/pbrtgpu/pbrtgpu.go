// Package pbrtgpu is the cgo binding a go-pbrt maintainer adds to call the
// MI355X hot path (include/pbrt_gpu.h, include/pbrt_scene.h) from Go.
//
// It replaces, frame-granular:
//   - pbrt.Render / renderWorker (pkg/pbrt/integrator.go:228-350) with
//     Renderer.RenderFrame (Path.Li and DirectLighting.Li run on the device);
//   - (*accelerator.BVH).Intersect / IntersectP (pkg/accelerator/bvh.go:659-765)
//     with Renderer.Intersect / IntersectP over ray batches;
//   - Film.WriteImage's pixel conversion (pkg/pbrt/film.go:142-179) with FilmToRGBA.
//
// The reference's constructors (internal/render/server.go:32-164) keep their
// parameters in unexported fields, so a scene is described through the
// SceneBuilder below, which mirrors them one call each.
//
// No Go toolchain exists in the build image of this repository: this file is
// not compiled here. tests/test_go_shim.py compiles its cgo preamble and every
// C identifier it uses against the headers with gcc.
package pbrtgpu

// #cgo CFLAGS: -I${SRCDIR}/../../../include
// #cgo LDFLAGS: -L${SRCDIR}/../../../go-pbrt_amd/lib -lpbrt_gpu -Wl,-rpath,${SRCDIR}/../../../go-pbrt_amd/lib
// #include <stdlib.h>
// #include "pbrt_gpu.h"
// #include "pbrt_scene.h"
import "C"

import (
	"context"
	"fmt"
	"image"
	"unsafe"
)

// ---------------------------------------------------------------- scenes

// SceneBuilder records a scene as server.go builds it (pbrt_sb_*).
type SceneBuilder struct {
	b    *C.pbrt_scene_builder
	desc *C.pbrt_scene_desc
}

// Transform is pbrt.Transform (transform.go:144): matrix and inverse.
type Transform = C.pbrt_transform

func NewSceneBuilder() *SceneBuilder { return &SceneBuilder{b: C.pbrt_sb_create()} }

// ReadmeScene is internal/render/server.go:32-164 at w x h.
func ReadmeScene(w, h int64) (*SceneBuilder, error) {
	var b *C.pbrt_scene_builder
	if rc := C.pbrt_scene_readme(C.int64_t(w), C.int64_t(h), &b); rc != C.PBRT_OK {
		return nil, fmt.Errorf("pbrt_scene_readme: status %d", int(rc))
	}
	return &SceneBuilder{b: b}, nil
}

func Translate(x, y, z float64) Transform {
	var t Transform
	C.pbrt_translate(C.double(x), C.double(y), C.double(z), &t)
	return t
}

func RotateX(deg float64) Transform {
	var t Transform
	C.pbrt_rotate_x(C.double(deg), &t)
	return t
}

func Mul(a, b Transform) Transform {
	var t Transform
	C.pbrt_transform_mul(&a, &b, &t)
	return t
}

func d3(v [3]float64) *C.double { return (*C.double)(unsafe.Pointer(&v[0])) }

// AddSphere is pbrt.NewSphereShape (sphere.go:19-35); returns the shape index.
func (s *SceneBuilder) AddSphere(o2w Transform, reverse bool, radius, zMin, zMax, phiMax float64) int {
	var sd C.pbrt_shape_desc
	rev := C.int(0)
	if reverse {
		rev = 1
	}
	C.pbrt_make_sphere(&o2w, rev, C.double(radius), C.double(zMin), C.double(zMax), C.double(phiMax), &sd)
	return int(C.pbrt_sb_add_shape(s.b, &sd))
}

// AddDisk is shapes.NewDisk (pkg/shapes/disk.go:22-35).
func (s *SceneBuilder) AddDisk(o2w Transform, height, radius, inner, phiMax float64) int {
	var sd C.pbrt_shape_desc
	C.pbrt_make_disk(&o2w, C.double(height), C.double(radius), C.double(inner), C.double(phiMax), &sd)
	return int(C.pbrt_sb_add_shape(s.b, &sd))
}

// AddMatte is materials.NewMatteMaterial with a constant Kd (sigma > 0: OrenNayar).
func (s *SceneBuilder) AddMatte(kd [3]float64, sigma float64) int {
	var m C.pbrt_material_desc
	C.pbrt_make_matte_constant(C.double(kd[0]), C.double(kd[1]), C.double(kd[2]), C.double(sigma), &m)
	return int(C.pbrt_sb_add_material(s.b, &m))
}

// AddCheckerMatte is NewMatteMaterial(textures.NewCheckerboard2D(NewPlanarMapping2D(vs, vt, ds, dt), tex1, tex2)).
func (s *SceneBuilder) AddCheckerMatte(vs, vt [3]float64, ds, dt float64, tex1, tex2 [3]float64, sigma float64) int {
	var m C.pbrt_material_desc
	C.pbrt_make_matte_checkerboard(d3(vs), d3(vt), C.double(ds), C.double(dt), d3(tex1), d3(tex2), C.double(sigma), &m)
	return int(C.pbrt_sb_add_material(s.b, &m))
}

// AddMirror is materials.NewMirror (mirror.go:9-14) with Kr.
func (s *SceneBuilder) AddMirror(kr [3]float64) int {
	var m C.pbrt_material_desc
	C.pbrt_make_mirror(d3(kr), &m)
	return int(C.pbrt_sb_add_material(s.b, &m))
}

// AddGlass is materials.NewGlass (glass.go:15-26) with constant textures.
func (s *SceneBuilder) AddGlass(kr, kt [3]float64, uRough, vRough, eta float64) int {
	var m C.pbrt_material_desc
	C.pbrt_make_glass(d3(kr), d3(kt), C.double(uRough), C.double(vRough), C.double(eta), &m)
	return int(C.pbrt_sb_add_material(s.b, &m))
}

// AddPrimitive is NewGeometricPrimitive, wrapped in NewTransformedPrimitive when
// primToWorld is non-nil (primitive.go:22-129).
func (s *SceneBuilder) AddPrimitive(shape, material int, primToWorld *Transform) int {
	var p C.pbrt_primitive_desc
	p.shape = C.int32_t(shape)
	p.material = C.int32_t(material)
	p.kind = C.PBRT_PRIM_GEOMETRIC
	if primToWorld != nil {
		p.kind = C.PBRT_PRIM_TRANSFORMED
		p.prim_to_world = *primToWorld
	}
	return int(C.pbrt_sb_add_primitive(s.b, &p))
}

// AddPointLight is lights.NewPointLight (point.go:19-30).
func (s *SceneBuilder) AddPointLight(l2w Transform, I [3]float64) int {
	var l C.pbrt_light_desc
	C.pbrt_make_point_light(&l2w, d3(I), &l)
	return int(C.pbrt_sb_add_light(s.b, &l))
}

// AddDistantLight is lights.NewDistantLight (distant.go:19-34).
func (s *SceneBuilder) AddDistantLight(l2w Transform, L, w [3]float64) int {
	var l C.pbrt_light_desc
	C.pbrt_make_distant_light(&l2w, d3(L), d3(w), &l)
	return int(C.pbrt_sb_add_light(s.b, &l))
}

// AddAreaLight is lights.NewDiffuseAreaLight (diffuse.go:19-34) over a sphere shape.
func (s *SceneBuilder) AddAreaLight(Lemit [3]float64, shape int, twoSided bool) int {
	var l C.pbrt_light_desc
	ts := C.int(0)
	if twoSided {
		ts = 1
	}
	C.pbrt_make_diffuse_area_light(d3(Lemit), C.int(shape), ts, &l)
	return int(C.pbrt_sb_add_light(s.b, &l))
}

// Build is accelerator.NewBVH(prims, maxPrimsInNode, SplitSAH) + pbrt.NewScene.
func (s *SceneBuilder) Build(maxPrimsInNode int) error {
	var d *C.pbrt_scene_desc
	if rc := C.pbrt_sb_build(s.b, C.int(maxPrimsInNode), &d); rc != C.PBRT_OK {
		return fmt.Errorf("pbrt_sb_build: status %d", int(rc))
	}
	s.desc = d
	return nil
}

func (s *SceneBuilder) Close() { C.pbrt_sb_destroy(s.b) }

// ------------------------------------------------------------- rendering

// PathDesc is integrator.NewPath(maxDepth, camera, sampler, ...) with
// sampler.NewStratified(xs, ys, jitter, nDims) (server.go:142-164).
func PathDesc(xs, ys int32, jitter bool, nDims, maxDepth int32, rrThreshold float64, strategy int32) C.pbrt_render_desc {
	var rd C.pbrt_render_desc
	rd.sampler_x, rd.sampler_y, rd.n_dims = C.int32_t(xs), C.int32_t(ys), C.int32_t(nDims)
	if jitter {
		rd.jitter = 1
	}
	rd.integrator = C.PBRT_INTEGRATOR_PATH
	rd.max_depth = C.int32_t(maxDepth)
	rd.rr_threshold = C.double(rrThreshold)
	rd.light_strategy = C.int32_t(strategy)
	rd.tile_size = 16
	rd.mode = C.PBRT_MODE_EXACT
	return rd
}

// WithRandomSampler switches rd to sampler.NewRandomSampler(ns, seed) (random.go:12-57).
func WithRandomSampler(rd *C.pbrt_render_desc, ns int32) { C.pbrt_random_sampler(C.int32_t(ns), rd) }

// Renderer owns a device-resident scene (one per GPU).
type Renderer struct {
	ctx  *C.pbrt_gpu_ctx
	w, h int // CroppedPixelBounds extent of the scene's film
}

func NewRenderer(s *SceneBuilder, device int) (*Renderer, error) {
	if s.desc == nil {
		return nil, fmt.Errorf("pbrtgpu: scene not built")
	}
	var opts C.pbrt_gpu_opts
	opts.device = C.int32_t(device)
	var ctx *C.pbrt_gpu_ctx
	if rc := C.pbrt_gpu_create(s.desc, &opts, &ctx); rc != C.PBRT_OK {
		return nil, fmt.Errorf("pbrt_gpu_create: status %d", int(rc))
	}
	f := s.desc.film
	return &Renderer{ctx: ctx, w: int(f.crop_max_x - f.crop_min_x), h: int(f.crop_max_y - f.crop_min_y)}, nil
}

// RenderFrame is pbrt.Render for one frame: film receives the merged XYZ sums
// Film.MergeFilmTile would hold, row-major W*H*3 float64. ctx cancellation maps
// to pbrt_gpu_cancel, as errgroup cancels the CPU workers (integrator.go:305-345).
func (r *Renderer) RenderFrame(ctx context.Context, rd *C.pbrt_render_desc, film []float64) error {
	if len(film) < r.w*r.h*3 || len(film) == 0 {
		return fmt.Errorf("pbrtgpu: film holds %d values, the frame needs %d", len(film), r.w*r.h*3)
	}
	if err := ctx.Err(); err != nil {
		return err
	}
	// pbrt_gpu_cancel acts on the render in flight only: a cancel that lands
	// before the render starts or after it ends is a no-op (include/pbrt_gpu.h)
	// The watcher is joined before RenderFrame returns: a cancel racing the end
	// of the render must not reach pbrt_gpu_cancel after the caller's Close
	// (pbrt_gpu_destroy frees the context the cancel locks).
	// a context cancelled before the frame starts renders nothing (the
	// reference's tile producer returns gtx.Err(), integrator.go:333-336)
	if err := ctx.Err(); err != nil {
		return err
	}
	done := make(chan struct{})
	exited := make(chan struct{})
	go func() {
		defer close(exited)
		select {
		case <-ctx.Done():
			C.pbrt_gpu_cancel(r.ctx)
		case <-done:
		}
	}()
	var st C.pbrt_gpu_stats
	rc := C.pbrt_gpu_render(r.ctx, rd, (*C.double)(unsafe.Pointer(&film[0])), &st)
	close(done)
	<-exited
	switch rc {
	case C.PBRT_OK:
		// the frame is complete: a cancel that reached the device while the
		// render was in flight returns PBRT_E_CANCELLED instead, and one that
		// came after the last kernel (or in the instant before the render was
		// in flight) leaves a valid film, as the reference's g.Wait() returns
		// nil once every tile was handed out (integrator.go:311-347)
		return nil
	case C.PBRT_E_CANCELLED:
		if err := ctx.Err(); err != nil {
			return err
		}
		return context.Canceled
	case C.PBRT_E_REF_PANIC: // the CPU reference panics here; keep that contract
		panic(fmt.Sprintf("go-pbrt panic kind %d at tile %d pixel (%d,%d) sample %d bounce %d",
			int(st.panic_kind), int(st.panic_tile), int64(st.panic_pixel_x), int64(st.panic_pixel_y),
			int(st.panic_sample), int(st.panic_bounce)))
	default:
		return fmt.Errorf("pbrt_gpu_render: %s", C.GoString(C.pbrt_gpu_last_error(r.ctx)))
	}
}

// Intersect is BVH.Intersect over a batch (rays and hits are caller-owned SoA).
func (r *Renderer) Intersect(rays *C.pbrt_ray_soa, n int, hits *C.pbrt_hit_soa) error {
	if rc := C.pbrt_gpu_intersect(r.ctx, rays, C.size_t(n), hits); rc != C.PBRT_OK {
		return fmt.Errorf("pbrt_gpu_intersect: %s", C.GoString(C.pbrt_gpu_last_error(r.ctx)))
	}
	return nil
}

// IntersectP is BVH.IntersectP over a batch; occluded[i] is 0 or 1.
func (r *Renderer) IntersectP(rays *C.pbrt_ray_soa, n int, occluded []uint8) error {
	if n <= 0 {
		return nil
	}
	if len(occluded) < n {
		return fmt.Errorf("pbrtgpu: %d results for %d rays", len(occluded), n)
	}
	if rc := C.pbrt_gpu_intersect_p(r.ctx, rays, C.size_t(n), (*C.uint8_t)(unsafe.Pointer(&occluded[0]))); rc != C.PBRT_OK {
		return fmt.Errorf("pbrt_gpu_intersect_p: %s", C.GoString(C.pbrt_gpu_last_error(r.ctx)))
	}
	return nil
}

func (r *Renderer) Close() { C.pbrt_gpu_destroy(r.ctx) }

// FilmToRGBA is Film.WriteImage's pixel loop (film.go:156-161): uint8(Clamp(v, 0, 1) * 255)
// of the XYZ sums, NaN -> 0, alpha 255; encode the result with image/png as WriteImage does.
func FilmToRGBA(film []float64, w, h int) (*image.RGBA, error) {
	if w <= 0 || h <= 0 || len(film) < w*h*3 {
		return nil, fmt.Errorf("pbrtgpu: film holds %d values, %dx%d needs %d", len(film), w, h, w*h*3)
	}
	img := image.NewRGBA(image.Rect(0, 0, w, h))
	if rc := C.pbrt_film_to_rgba8((*C.double)(unsafe.Pointer(&film[0])), C.int64_t(w), C.int64_t(h),
		(*C.uint8_t)(unsafe.Pointer(&img.Pix[0]))); rc != C.PBRT_OK {
		return nil, fmt.Errorf("pbrt_film_to_rgba8: status %d", int(rc))
	}
	return img, nil
}
