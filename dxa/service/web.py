"""Single-page operations console served at ``/`` — a compact stand-in for the reference's React website
(Website/Packages/datax-pipeline: flow list/editor, jobs page, query editor with LiveQuery, metrics dashboard).

Plain HTML + fetch against the same REST routes; no build step, no external assets (the box has no network)."""

INDEX_HTML = r"""<!doctype html>
<html><head><meta charset="utf-8"><title>dxa console</title>
<style>
body{font-family:system-ui,sans-serif;margin:0;background:#f4f5f7;color:#222}
header{background:#1b2a3a;color:#fff;padding:10px 18px;font-size:18px}
nav button{margin-right:6px}
main{display:grid;grid-template-columns:320px 1fr;gap:14px;padding:14px}
section{background:#fff;border-radius:6px;padding:12px;box-shadow:0 1px 2px #0002}
table{border-collapse:collapse;width:100%;font-size:13px}td,th{border-bottom:1px solid #eee;padding:4px;text-align:left}
textarea{width:100%;height:160px;font-family:monospace;font-size:12px}
pre{background:#111;color:#cfc;padding:8px;max-height:300px;overflow:auto;font-size:12px}
canvas{width:100%;height:180px;background:#fafafa;border:1px solid #ddd}
.err{color:#b00}
</style></head><body>
<header>dxa — MI355X streaming ETL console</header>
<main>
<section><h3>Flows</h3><table id="flows"></table>
<h3>Jobs</h3><table id="jobs"></table><button onclick="refresh()">refresh</button></section>
<section>
<h3>Flow definition</h3>
<textarea id="flowjson" placeholder='{"name":"myflow","gui":{...}}'></textarea>
<nav><button onclick="saveFlow()">save</button><button onclick="flowOp('flow/generateconfigs')">generate</button>
<button onclick="flowOp('flow/startjobs')">start</button><button onclick="flowOp('flow/stopjobs')">stop</button>
<button onclick="flowOp('flow/restartjobs')">restart</button><button onclick="flowOp('flow/delete')">delete</button></nav>
<h3>Live query</h3>
<textarea id="query" placeholder="--DataXQuery--&#10;T1 = SELECT * FROM DataXProcessedInput"></textarea>
<nav><button onclick="newKernel()">new kernel</button><button onclick="execQuery()">execute</button>
<span id="kernel"></span></nav>
<h3>Metrics</h3><input id="metric" size="50" placeholder="DATAX-myflow:Input_DataXProcessedInput_Events_Count">
<button onclick="pollMetric()">plot</button><canvas id="chart" width="900" height="180"></canvas>
<pre id="out"></pre>
</section></main>
<script>
let kernelId=null, current=null;
async function api(route, body){const r=await fetch('/api/'+route,{method:'POST',headers:{'Content-Type':'application/json'},
  body:JSON.stringify(body===undefined?{}:body)});const j=await r.json();
  document.getElementById('out').textContent=JSON.stringify(j,null,1).slice(0,20000);return j;}
async function refresh(){const f=await api('flow/getall/min');const t=document.getElementById('flows');
  t.innerHTML='<tr><th>name</th><th>owner</th></tr>'+(f.result||[]).map(x=>`<tr><td><a href="#" onclick="loadFlow('${x.name}')">${x.name}</a></td><td>${x.owner}</td></tr>`).join('');
  const j=await api('job/getall');document.getElementById('jobs').innerHTML='<tr><th>job</th><th>state</th></tr>'+
  (j.result||[]).map(x=>`<tr><td>${x.name}</td><td>${x.state}</td></tr>`).join('');}
async function loadFlow(n){current=n;const f=await api('flow/get',{name:n});
  document.getElementById('flowjson').value=JSON.stringify(f.result,null,1);}
async function saveFlow(){const f=JSON.parse(document.getElementById('flowjson').value);current=f.name;await api('flow/save',f);refresh();}
async function flowOp(op){if(current)await api(op,{name:current});refresh();}
async function newKernel(){const r=await api('kernel',{flowName:current});kernelId=r.result;
  document.getElementById('kernel').textContent=kernelId?('kernel '+kernelId.slice(0,8)):'';}
async function execQuery(){if(kernelId)await api('kernel/executequery',{kernelId,query:document.getElementById('query').value});}
async function pollMetric(){const m=document.getElementById('metric').value;const now=Date.now();
  const r=await fetch(`/api/metrics/get?m=${encodeURIComponent(m)}&s=${now-3600e3}&e=${now}`);const pts=await r.json();
  const c=document.getElementById('chart'),g=c.getContext('2d');g.clearRect(0,0,c.width,c.height);if(!pts.length)return;
  const xs=pts.map(p=>p.uts),ys=pts.map(p=>+p.val),x0=Math.min(...xs),x1=Math.max(...xs)||1,y1=Math.max(...ys)||1;
  g.beginPath();pts.forEach((p,i)=>{const x=(p.uts-x0)/(x1-x0||1)*(c.width-20)+10,y=c.height-10-(+p.val)/y1*(c.height-20);
  i?g.lineTo(x,y):g.moveTo(x,y);});g.strokeStyle='#2a6';g.stroke();g.fillText(y1.toFixed(1),2,10);}
refresh();
</script></body></html>
"""
