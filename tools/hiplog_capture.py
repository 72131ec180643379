"""Filter an AMD_LOG_LEVEL=3 HIP API log down to the stream / event calls of the LAST capture
(hipStreamBeginCapture onward): hipEventRecord, hipStreamWaitEvent, hipStreamBeginCapture /
EndCapture, and reconstruct which streams joined the capture through which stream.

    python tools/hiplog_capture.py LOG > summary.txt
"""
import re
import sys


def main(path):
    lines = open(path, errors='replace').read().splitlines()
    start = max((i for i, l in enumerate(lines) if 'hipStreamBeginCapture (' in l), default=0)
    keep = [l for l in lines[start:] if re.search(r'(hipEventRecord|hipStreamWaitEvent|hipStreamBeginCapture|'
                                                  r'hipStreamEndCapture) \(', l)]
    ev_stream = {}
    joined = {}
    origin = None
    for l in keep:
        args = re.search(r'\((.*)\)', l).group(1)
        ptrs = re.findall(r'0x[0-9a-f]+', args)
        if 'hipStreamBeginCapture' in l and ptrs:
            origin = ptrs[0]
            joined[origin] = None
        elif 'hipEventRecord' in l and len(ptrs) >= 2:
            ev_stream[ptrs[0]] = ptrs[1]
        elif 'hipEventRecord' in l and len(ptrs) == 1:
            ev_stream[ptrs[0]] = '0x0'
        elif 'hipStreamWaitEvent' in l and len(ptrs) >= 2:
            s, e = ptrs[0], ptrs[1]
            src = ev_stream.get(e)
            if s not in joined and src in joined:
                joined[s] = src
                print(f'JOIN {s} via event {e} recorded on {src}' + ('' if src == origin else '   <-- NESTED'))
    print(f'origin {origin}; {len(keep)} stream/event calls in the capture; joined: {joined}')
    end = next((i for i in range(start, len(lines)) if 'hipStreamEndCapture (' in lines[i]), len(lines))
    cap = lines[start:end]
    mem = [l for l in cap if re.search(r'hipMemset\w* \(|hipMemcpy\w* \(', l)]
    print(f'{len(mem)} memset / memcpy calls inside the capture:')
    for l in mem[:60]:
        print('  ', l[l.find('hip'):][:160])
    from collections import Counter
    launches = Counter()
    for l in cap:
        m = re.search(r'(hip\w*Launch\w*) \(.*?stream:(0x[0-9a-f]+|<null>)', l)
        if m:
            launches[(m.group(1), m.group(2))] += 1
    print('kernel launches inside the capture by (API, stream):')
    for (api, st), n in sorted(launches.items(), key=lambda kv: -kv[1]):
        print(f'   {api:28s} {st:16s} {n:6d}' + ('' if st in joined else '   <-- NOT A CAPTURE STREAM'))
    for l in keep[-40:]:
        print(l[l.find('hip'):][:200])
    # the first API call of the capture that did not return hipSuccess, with the calls before it
    for i in range(start, len(lines)):
        if 'Returned hip' in lines[i] and 'Returned hipSuccess' not in lines[i] and 'hipErrorNotReady' not in lines[i]:
            print('\nFIRST ERROR in the capture:')
            for l in lines[max(start, i - 40):i + 1]:
                print(l[l.find('hip') if 'hip' in l else 0:][:220])
            # the events the last stream waits before the error waited on: where were they recorded?
            waits = [l for l in lines[start:i] if 'hipStreamWaitEvent (' in l][-3:]
            for w in waits:
                e = re.findall(r'event:(0x[0-9a-f]+)', w)
                if not e:
                    continue
                rec = [j for j in range(start, i) if 'hipEventRecord (' in lines[j] and e[0] in lines[j]]
                print('\nWAIT', w[w.find('hip'):][:150])
                if rec:
                    j = rec[-1]
                    print('  recorded at', lines[j][lines[j].find('hip'):][:150])
                    print('  API calls around that record:')
                    for l in lines[max(start, j - 25):j + 3]:
                        if ' ( ' in l:
                            print('    ', l[l.find('hip'):][:160])
            break


if __name__ == '__main__':
    main(sys.argv[1])
