// Host C++ API of the MI355X volume renderer: a header-only mirror of the reference's classes
// (wantonsushi/3DG-vol-renderer include/*.h) on top of the C ABI in include/vr_hip.h.
//
//   Scene scene = Scene::load_GMM("scenes/gaussians/many_gaussians.txt");     // scene.h:72-120
//   auto camera = std::make_shared<Pinhole_Camera>(pos, view_dir, fov);        // camera.h:31-54
//   Image image(512, 512);                                                     // image.h:9-20
//   auto integrator = std::make_unique<RayMarchingGaussians>(camera);          // test_integrators.h:143
//   integrator->render(scene, image);                                          // integrator.h:56
//   image.make_PPM("output.ppm");                                              // image.h:62-84
//
// Same class names, constructor arguments, public members and error behaviour
// (std::runtime_error). Rendering runs on the GPU through libvr_hip.so; there is no CPU renderer
// here. Link with -lvr_hip.
#pragma once

#include "camera.h"
#include "gaussian.h"
#include "gif.h"
#include "gmm.h"
#include "image.h"
#include "integrator.h"
#include "inverse_integrator.h"
#include "optimizer.h"
#include "ray.h"
#include "scene.h"
#include "smm.h"
#include "test_integrators.h"
