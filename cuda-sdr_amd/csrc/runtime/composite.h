// Composite graphs: the FilterDriver (a filter graph driven from inside a
// Filter, reference src/driver/FilterDriver.cpp), its JSON "Component" factory
// (src/driver/FilterDriverFactory.cpp:27-178), the port-remapping sink / source that expose inner
// ports (src/filters/PortRemappingSink.cpp, PortRemappingSource.cpp), the RF -> PCM audio component
// (src/filters/factories/RfToPcmAudioFactory.cpp:152-317) and the read-byte-count monitor
// (src/filters/ReadByteCountMonitor.cpp, §8f row 4).
#pragma once

#include <gpusdrpipeline/Factories.h>

#include <cstddef>
#include <vector>

namespace gsdr_rt {

// Low-pass FIR design for the RF -> PCM component. The reference designs with Parks-McClellan
// (remez, an un-vendored dependency) at the fred harris length estimate
// ceil(-dbAttenuation / (22 * transitionWidth / sampleRate)) (RfToPcmAudioFactory.cpp:44-47;
// dbAttenuation is negative dB there). This build uses that length with a Kaiser window
// (beta from |dbAttenuation|) around cutoff + transitionWidth / 2, unit DC gain, computed in double
// and rounded to float. Tap VALUES are therefore not the reference's (parity unpinned); the graph
// built around them is.
Status designLowPass(double sampleRate, double cutoff, double transitionWidth, double dbAttenuation,
                     std::vector<float>& taps) noexcept;

IFilterDriverFactory* newFilterDriverFactory(IFactories* factories) noexcept;

class SteppingDriver;
// The stepping driver inside a component (FilterDriver), or nullptr if `driver` is not one.
SteppingDriver* componentSteppingDriver(IDriver* driver) noexcept;
IPortRemappingSinkFactory* newPortRemappingSinkFactory() noexcept;
IPortRemappingSourceFactory* newPortRemappingSourceFactory() noexcept;
IRfToPcmAudioFactory* newRfToPcmAudioFactory(IFactories* factories) noexcept;
IReadByteCountMonitorFactory* newReadByteCountMonitorFactory() noexcept;

}  // namespace gsdr_rt
