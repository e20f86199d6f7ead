window.Plotly = {
  version: '2.0.0',
  toImage: function (fig, opts) {
    var meta = fig.layout.meta;
    var bin = atob(meta.mp3);
    var buf = new Uint8Array(bin.length);
    for (var i = 0; i < bin.length; i++) buf[i] = bin.charCodeAt(i);
    var ctx = new OfflineAudioContext(meta.nch || 2, 44100, meta.sr);
    return new Promise(function (resolve) {
      ctx.decodeAudioData(buf.buffer, function (ab) {
        var chans = [];
        for (var c = 0; c < ab.numberOfChannels; c++) {
          var d = ab.getChannelData(c);
          var u8 = new Uint8Array(d.buffer, d.byteOffset, d.byteLength);
          var s = '';
          for (var j = 0; j < u8.length; j += 8192) s += String.fromCharCode.apply(null, u8.subarray(j, j + 8192));
          chans.push(btoa(s));
        }
        resolve(JSON.stringify({sr: ab.sampleRate, len: ab.length, nch: ab.numberOfChannels, ch: chans}));
      }, function (e) { resolve(JSON.stringify({error: String(e)})); });
    });
  }
};
