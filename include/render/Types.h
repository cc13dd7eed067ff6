// render/Types.h — RenderSettings with its dirty flag, restated from the reference
// (libs/render/include/render/Types.h:43-95, libs/render/src/RenderSettings.cpp:5-54).
// Only width/height/isDirty/clearDirty drive the reference integrator (CPUPathTracer.cpp:132-149);
// the other fields are carried for interface parity.
#pragma once

#include <cstdint>

namespace render {

    class RenderSettings {
    public:
        RenderSettings() = default;

        void setResolution(uint32_t width, uint32_t height);
        void setProgressive(bool progressive);
        void setSamplesPerPixel(uint32_t samples);
        void setMaxBounces(uint32_t bounces);
        void setRussianRouletteDepth(uint32_t depth);
        void setExposure(float exposure);
        void setAutoExposure(bool enabled, float target_luminance = 0.18f);

        uint32_t getWidth() const { return m_width; }
        uint32_t getHeight() const { return m_height; }
        bool getProgressive() const { return m_progressive; }
        uint32_t getSamplesPerPixel() const { return m_samplesPerPixel; }
        uint32_t getMaxBounces() const { return m_maxBounces; }
        uint32_t getRussianRouletteDepth() const { return m_russianRouletteDepth; }
        float getExposure() const { return m_exposure; }
        bool getAutoExposure() const { return m_autoExposure; }
        float getTargetLuminance() const { return m_targetLuminance; }

        bool isDirty() const { return m_dirty; }
        void clearDirty() { m_dirty = false; }

    private:
        uint32_t m_width = 512;
        uint32_t m_height = 512;
        bool m_progressive = true;
        uint32_t m_samplesPerPixel = 64;
        uint32_t m_maxBounces = 8;
        uint32_t m_russianRouletteDepth = 3;
        float m_exposure = 1.0f;
        bool m_autoExposure = false;
        float m_targetLuminance = 0.18f;
        bool m_dirty = true;  // dirty on construction

        void markDirty() { m_dirty = true; }
    };

}
