// vol_render: command-line renderer over the C++ host API (the role of the reference's
// tests/main.cpp, which hard-codes scene, camera and integrator; here they are arguments).
//
//   vol_render --scene scenes/many_gaussians.txt [--spheres] [--xml] [--size 512x512]
//              [--integrator gaussians|pure|spheres|test|freeflight|multiscatter] [--step 0.01] [--env 20]
//              [--spp N] (free-flight paths per pixel; main.cpp:42 renders MultiScatterGaussians at 256)
//              [--camera pinhole|ortho] [--pos 0,1,6] [--lookat 0,1,0] [--fov 0.785398]
//              [--out output.ppm] [--dump-rays N] [--devices 0,1,...]
//
// --record (multiscatter): the 3-argument render with per-pixel Gaussian lists (RECORD_PIXEL_GAUSSIANS);
// prints the number of recorded (pixel, Gaussian) pairs.
// --inverse N --ref I_ref.ppm [--seed S] [--stoch K] [--lr X] [--final-spp F] [--sfd-out DIR]: N iterations
// of StochasticFiniteDiffInverseIntegrator from --scene towards I_ref (MultiScatterGaussians at --spp);
// prints every iteration's mean loss (the reference's tests/main.cpp inverse mode, main.cpp:48-75).
// --gif out.gif [--frames 120] [--fps 30]: the reference driver's turntable (main.cpp:81-114): an
// Orthographic_Camera orbiting the look-at point at radius 6 and height +1, RayMarchingGaussians
// (step 0.01, --env samples), one GIF frame each.
// --devices renders on a multi-GPU context over exactly these GPUs (tiles split, RCCL gather); by
// default every visible GPU is used (one GPU: a plain single-device context).
// --dump-rays N prints the first N primary rays (host only, no GPU) — used by the CPU tests.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <cmath>
#include <numbers>
#include <string>
#include <vector>

#include "vr/integrator.h"
#include "vr/gif.h"
#include "vr/inverse_integrator.h"
#include "vr/test_integrators.h"

static Eigen::Vector3f parse3(const char* s) {
    float a = 0, b = 0, c = 0;
    if (std::sscanf(s, "%f,%f,%f", &a, &b, &c) != 3) throw std::runtime_error(std::string("bad vector: ") + s);
    return Eigen::Vector3f(a, b, c);
}

int main(int argc, char** argv) try {
    std::string scene_path, out = "output.ppm", integ = "gaussians", cam_type = "pinhole";
    bool spheres = false, xml = false;
    unsigned W = 512, H = 512;
    float step = 0.01f, fov = 0.25f * std::numbers::pi_v<float>;
    int env = -1, dump = 0, spp = -1;
    std::vector<int> devices;
    bool record = false;
    int inverse = 0, stoch = 4, final_spp = 0;
    uint64_t seed = 0;
    float lr = 1e-2f;
    std::string ref_path, sfd_out, gif_path;
    int frames = 120;
    float fps = 30.0f;
    Eigen::Vector3f pos(0, 1, 6), lookat(0, 1, 0);
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&]() -> const char* {
            if (i + 1 >= argc) throw std::runtime_error("missing value for " + a);
            return argv[++i];
        };
        if (a == "--scene") scene_path = next();
        else if (a == "--spheres") spheres = true;
        else if (a == "--xml") xml = true;
        else if (a == "--size") { if (std::sscanf(next(), "%ux%u", &W, &H) != 2) throw std::runtime_error("bad --size"); }
        else if (a == "--integrator") integ = next();
        else if (a == "--spp") spp = std::stoi(next());
        else if (a == "--step") step = std::strtof(next(), nullptr);
        else if (a == "--env") env = std::atoi(next());
        else if (a == "--camera") cam_type = next();
        else if (a == "--pos") pos = parse3(next());
        else if (a == "--lookat") lookat = parse3(next());
        else if (a == "--fov") fov = std::strtof(next(), nullptr);
        else if (a == "--out") out = next();
        else if (a == "--dump-rays") dump = std::atoi(next());
        else if (a == "--record") record = true;
        else if (a == "--gif") gif_path = next();
        else if (a == "--frames") frames = std::atoi(next());
        else if (a == "--fps") fps = std::strtof(next(), nullptr);
        else if (a == "--inverse") inverse = std::atoi(next());
        else if (a == "--ref") ref_path = next();
        else if (a == "--seed") seed = std::strtoull(next(), nullptr, 10);
        else if (a == "--stoch") stoch = std::atoi(next());
        else if (a == "--lr") lr = std::strtof(next(), nullptr);
        else if (a == "--final-spp") final_spp = std::atoi(next());
        else if (a == "--sfd-out") sfd_out = next();
        else if (a == "--devices") {
            std::string v = next();
            for (size_t p = 0; p <= v.size();) {
                size_t q = v.find(',', p);
                if (q == std::string::npos) q = v.size();
                devices.push_back(std::stoi(v.substr(p, q - p)));
                p = q + 1;
            }
        }
        else throw std::runtime_error("unknown argument " + a);
    }
    if (scene_path.empty()) throw std::runtime_error("--scene is required");

    std::shared_ptr<Camera> camera;
    Scene scene;
    vr_render_params xml_params{};
    if (xml) {
        vr_camera st{};
        uint32_t w = 0, h = 0;
        scene = Scene::load_XML(scene_path, &st, &w, &h, &xml_params);
        camera = std::make_shared<State_Camera>(st);
        W = w;
        H = h;
        integ = xml_params.integrator == VR_RAYMARCH_SPHERES ? "spheres" : "gaussians";
        if (env < 0) env = xml_params.env_samples;
        step = xml_params.step_size;
    } else {
        scene = spheres ? Scene::load_SMM(scene_path) : Scene::load_GMM(scene_path);
        Eigen::Vector3f view_dir = (lookat - pos).normalized();
        if (cam_type == "ortho") camera = std::make_shared<Orthographic_Camera>(pos, view_dir);
        else camera = std::make_shared<Pinhole_Camera>(pos, view_dir, fov);
    }
    std::printf("scene: %zu primitives, %zu lights\n", scene.get_num_primitives(), scene.lights.size());

    if (dump > 0) {  // host-only: primary rays through pixel centres, row-major
        for (int k = 0; k < dump; ++k) {
            unsigned x = k % W, y = k / W;
            Eigen::Vector2d uv((x + 0.5) / W, (y + 0.5) / H);
            Ray r = camera->sample_ray(uv);
            std::printf("ray %u %u %.9g %.9g %.9g %.9g %.9g %.9g\n", x, y, r.origin.x(), r.origin.y(), r.origin.z(),
                        r.direction.x(), r.direction.y(), r.direction.z());
        }
        return 0;
    }

    if (!gif_path.empty()) {  // main.cpp:81-114
        const float radius = 6.0f, height_pos = 1.0f;
        GifWriter gif;
        if (!GifBegin(&gif, gif_path.c_str(), W, H, (uint32_t)(100.0f / fps))) throw std::runtime_error(vr_last_error());
        for (int frame = 0; frame < frames; ++frame) {
            const float angle = 2.0f * std::numbers::pi_v<float> * ((float)frame / (float)frames);
            Eigen::Vector3f cpos = lookat + Eigen::Vector3f(radius * std::sin(angle), height_pos, radius * std::cos(angle));
            Eigen::Vector3f vd = (lookat - cpos).normalized();
            auto cam = std::make_shared<Orthographic_Camera>(cpos, vd);
            RayMarchingGaussians rm(cam, step, env < 0 ? 20 : env);
            if (!devices.empty()) rm.set_devices(devices);
            Image image(W, H);
            rm.render(scene, image);
            auto rgba = image.get_rgba_buffer();
            if (!GifWriteFrame(&gif, rgba.data(), W, H, (uint32_t)(100.0f / fps))) throw std::runtime_error(vr_last_error());
            std::printf("Frame %d / %d complete.\n", frame + 1, frames);
        }
        if (!GifEnd(&gif)) throw std::runtime_error(vr_last_error());
        std::printf("GIF saved.\n");
        return 0;
    }

    std::unique_ptr<HipIntegrator> integrator;
    if (integ == "gaussians") integrator = std::make_unique<RayMarchingGaussians>(camera, step, env < 0 ? 20 : env);
    else if (integ == "spheres") integrator = std::make_unique<RayMarchingSpheres>(camera, step, env < 0 ? 5 : env);
    else if (integ == "pure") integrator = std::make_unique<PureRayMarching>(camera, step, env < 0 ? 20 : env);
    else if (integ == "test") integrator = std::make_unique<TestIntegrator>(camera);
    else if (integ == "freeflight") integrator = std::make_unique<FreeFlightGaussians>(camera, spp < 0 ? 256 : spp);
    else if (integ == "multiscatter") integrator = std::make_unique<MultiScatterGaussians>(camera, spp < 0 ? 16 : spp);
    else throw std::runtime_error("unknown integrator " + integ);

    if (!devices.empty()) integrator->set_devices(devices);
    if (inverse > 0) {  // main.cpp:48-75: optimise the scene towards a reference image
        if (integ != "multiscatter") throw std::runtime_error("--inverse needs --integrator multiscatter");
        Image I_ref(ref_path);
        auto fwd = std::make_shared<MultiScatterGaussians>(camera, spp < 0 ? 16 : spp);
        if (!devices.empty()) fwd->set_devices(devices);
        SFDDConfig cfg;
        cfg.max_iters = inverse;
        cfg.num_stoch_samples = stoch;
        cfg.lr = lr;
        cfg.seed = seed;
        cfg.final_samples = final_spp;
        cfg.out_dir = sfd_out;
        StochasticFiniteDiffInverseIntegrator sfd(camera, fwd, cfg);
        if (!sfd.optimize(scene, I_ref)) throw std::runtime_error("SFD optimisation failed");
        for (size_t i = 0; i < sfd.loss_history().size(); ++i) std::printf("sfd iter %zu loss %.17g\n", i, sfd.loss_history()[i]);
        if (final_spp > 0) std::printf("sfd final loss %.17g\n", sfd.final_loss());
        return 0;
    }
    Image image(W, H);
    auto t0 = std::chrono::high_resolution_clock::now();
    if (record) {
        auto* ms = dynamic_cast<MultiScatterGaussians*>(integrator.get());
        if (!ms) throw std::runtime_error("--record needs --integrator multiscatter");
        std::vector<std::vector<uint32_t>> per_pixel;
        ms->render(scene, image, &per_pixel);
        size_t pairs = 0;
        for (const auto& l : per_pixel) pairs += l.size();
        std::printf("recorded pairs %zu\n", pairs);
    } else {
        integrator->render(scene, image);
    }
    auto t1 = std::chrono::high_resolution_clock::now();
    vr_render_stats st = integrator->stats();
    std::printf("Render time: %.6f seconds (device %.3f ms, %lld pixels, %lld fallback, %d device(s)%s)\n",
                std::chrono::duration<double>(t1 - t0).count(), st.kernel_ms, (long long)st.pixels,
                (long long)st.fallback_pixels, vr_ctx_num_devices(integrator->context()),
                !vr_ctx_uses_rccl(integrator->context()) ? ""
                : vr_ctx_num_devices(integrator->context()) > 1 ? ", RCCL gather"
                                                                : ", RCCL communicator (one rank: nothing to gather)");
    image.make_PPM(out);
    return 0;
} catch (const std::exception& e) {
    std::fprintf(stderr, "vol_render: %s\n", e.what());
    return 1;
}
