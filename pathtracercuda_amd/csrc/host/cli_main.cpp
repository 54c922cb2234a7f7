// `pathtracer` command line tool: the reference's headless renderer (src/main.cpp:22-295) on
// MI355X.  Same options, defaults, messages and output semantics; additions:
//   -gpus N        tile the image over N GPUs (rows interleaved; bit-identical to 1 GPU)
//   -chunk N       samples per render() call of the headless loop (default 8, main.cpp:272)
//   -single_launch run all render() calls of the loop in one kernel launch (bit-identical)
// The windowed / interactive mode (-window, -enable_controls) is not supported.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <thread>
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
        printf("%-30s Render on N GPUs (image rows interleaved)\n", "-gpus");
        printf("%-30s Samples per render() call (default 8)\n", "-chunk");
        printf("%-30s Run all render() calls in one kernel launch\n", "-single_launch");
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
    std::vector<std::unique_ptr<Pathtracer>> tiles;
    std::vector<Camera> cams;
    for (int g = 0; g < gpus; ++g) {
        tiles.emplace_back(new Pathtracer(params.m_width, params.m_height, g, (uint32_t)g, (uint32_t)gpus));
        cams.push_back(loadScene(*tiles.back(), params));
    }

    const uint32_t chunk = params.m_chunk;
    std::vector<float> gpuTime(gpus, 0.0f);
    auto renderTile = [&](int g) {
        Pathtracer& pt = *tiles[g];
        if (params.m_singleLaunch && params.m_spp > 0) {
            const uint32_t full = params.m_spp / chunk, rest = params.m_spp % chunk;
            if (full) { pt.renderChunks(cams[g], chunk, full, true); gpuTime[g] += pt.getTiming(); }
            if (rest) { pt.renderChunks(cams[g], rest, 1, full == 0); gpuTime[g] += pt.getTiming(); }
            return;
        }
        for (uint32_t i = 0; i < params.m_spp; i += chunk) {
            const uint32_t spp = std::min(i + chunk, params.m_spp) - i;
            pt.render(cams[g], spp, i == 0);
            gpuTime[g] += pt.getTiming();
            if (g == 0 && i % (chunk * 4) == 0) printf("Accumulated %d samples\n", (int)i);
        }
    };
    if (gpus == 1) renderTile(0);
    else {
        std::vector<std::thread> th;
        for (int g = 0; g < gpus; ++g) th.emplace_back(renderTile, g);
        for (auto& t : th) t.join();
    }
    const float totalGpuTime = *std::max_element(gpuTime.begin(), gpuTime.end());
    printf("Finished accumulating %d samples in %f ms GPU time\n", (int)params.m_spp, totalGpuTime);

    if (params.m_outputFilepath) {
        printf("Writing result to %s\n", params.m_outputFilepath);
        const uint32_t W = params.m_width, H = params.m_height;
        bool ok;
        if (params.m_outputHdr) {
            std::vector<float> img((size_t)W * H * 4);
            for (int g = 0; g < gpus; ++g) {
                const float* t = tiles[g]->getHDRImageData();
                for (uint32_t k = 0; k < tiles[g]->localRows(); ++k)
                    memcpy(&img[(size_t)(g + k * gpus) * W * 4], t + (size_t)k * W * 4, (size_t)W * 4 * sizeof(float));
            }
            ok = ptamd::writeHDR(params.m_outputFilepath, W, H, img.data(), true);
        } else {
            std::vector<uint8_t> img((size_t)W * H * 4);
            for (int g = 0; g < gpus; ++g) {
                const char* t = tiles[g]->getImageData();
                for (uint32_t k = 0; k < tiles[g]->localRows(); ++k)
                    memcpy(&img[(size_t)(g + k * gpus) * W * 4], t + (size_t)k * W * 4, (size_t)W * 4);
            }
            ok = ptamd::writePNG(params.m_outputFilepath, W, H, img.data(), true);
        }
        if (!ok) printf("Failed to write file!\n");
    }
    return EXIT_SUCCESS;
}
